#!/bin/bash
# Interleaved A/B of ILU env knobs on scripts/bench_ilu0.py (fp64 only).
#   SET=dc1,G2_circuit ROUNDS=2 bash scripts/env_ab.sh TAG "name:VAR=v VAR2=w" "name2:VAR=u" ...
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=$1; shift
O=gpurun_out/$TAG
mkdir -p "$O"
export TMPDIR=/tmp
SET=${SET:-thermomech_TK,G2_circuit,dc1,matrix-new_3}
for r in $(seq 1 "${ROUNDS:-2}"); do
    for spec in "$@"; do
        name=${spec%%:*}; envs=${spec#*:}
        env $envs timeout -k 10 300 python scripts/bench_ilu0.py --set "$SET" --fp64-only --reps 5 \
            > "$O/${name}_$r.txt" 2> "$O/${name}_$r.err" || { tail -20 "$O/${name}_$r.err"; exit 1; }
        echo "$name round $r: $(grep TOTAL "$O/${name}_$r.txt" | cut -c1-60)"
        cut -c1-16,50-68 "$O/${name}_$r.txt" | sed -n '2,$p' | grep -v "^median\|^TOTAL"
    done
done
