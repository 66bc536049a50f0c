#!/bin/bash
# ILU analysis wall time A/B (config 3, 21 matrices, 3 calls each; phases
# with RSP_ILU_TIMING=1): env variants interleaved, one process each.
#   bash scripts/an_ab.sh TAG "name:VAR=v ..." ...
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=$1; shift
O=gpurun_out/$TAG
mkdir -p "$O"
export TMPDIR=/tmp
for r in $(seq 1 "${ROUNDS:-1}"); do
    for spec in "$@"; do
        name=${spec%%:*}; envs=${spec#*:}
        env RSP_ILU_TIMING=1 $envs timeout -k 10 300 python scripts/ilu_analysis_timing.py moderate 3 \
            > "$O/${name}_$r.txt" 2>&1 || { tail -20 "$O/${name}_$r.txt"; exit 1; }
        echo "$name round $r: $(tail -1 "$O/${name}_$r.txt")"
        python3 - "$O/${name}_$r.txt" <<'PY'
import re, sys, collections
ph = collections.OrderedDict()
lines = open(sys.argv[1]).read().splitlines()
# phases of the 3rd call of every matrix: the last 5 phase lines before each "<name>: analysis" line
calls = collections.defaultdict(list)
cur = []
for l in lines:
    m = re.match(r"rsp_ilu0_analysis n=\d+ (.+?)\s+([\d.]+) ms", l)
    if m:
        cur.append((m.group(1).strip(), float(m.group(2))))
    elif ": analysis" in l:
        calls[l.split(":")[0]].append(cur)
        cur = []
for k in range(3):
    tot = collections.OrderedDict()
    for name, cs in calls.items():
        if len(cs) > k:
            for p, v in cs[k]:
                tot[p] = tot.get(p, 0.0) + v
    print(f"  call {k + 1}: " + ", ".join(f"{p} {v:.1f}" for p, v in tot.items()))
PY
    done
done
