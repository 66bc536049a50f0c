#!/bin/bash
# Round 4: ILU tests, then the narrow-pairs solve A/B and the analysis
# overlap A/B (previous library vs current).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/${1:-r4ov}
mkdir -p "$O"
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_ilu0.py tests/test_gpu_drivers.py -q -x -rf --timeout 300 --timeout-method thread > "$O/pytest.log" 2>&1
rc=$?; tail -2 "$O/pytest.log"; [ $rc -eq 0 ] || exit $rc
ROUNDS=2 bash scripts/env_ab.sh ${1:-r4ov}/pairs "def:X=0" "pairs:RSP_ILU_NARROW_PAIRS=1" "pairs3:RSP_ILU_NARROW_PAIRS=1 RSP_ILU_NARROW_WAVES=3" "fpairs:RSP_ILU_FNARROW_PAIRS=1" "both:RSP_ILU_FNARROW_PAIRS=1 RSP_ILU_NARROW_PAIRS=1" || exit 1
ROUNDS=2 bash scripts/an_ab.sh ${1:-r4ov}/an "cur:X=0" "prev:RSP_PROBE_LIB=$PWD/respasol_amd/build/ab/prev/librsp.so" || exit 1
RSP_ILU_TIMING=2 timeout -k 10 300 python scripts/ilu_analysis_timing.py moderate 2 > "$O/an_t2.txt" 2>&1 || exit 1
python3 - "$O/an_t2.txt" <<'PY'
import re, sys, collections
t = collections.defaultdict(float)
for l in open(sys.argv[1]):
    m = re.match(r"rsp_ilu0_analysis n=\d+\s+plan (\w+)\s+([\d.]+) ms", l)
    if m: t[m.group(1)] += float(m.group(2))
print("plan wall sums over both calls:", dict(t))
PY
