#!/bin/bash
# Round 4: ILU GPU tests, then config-3 timing: round-3 library vs the current
# one with dynamic (mode 0) and static (mode 1) flow claims.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=${1:-r4ilu3}
O=gpurun_out/$TAG
mkdir -p "$O"
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_gpu_ilu0.py tests/test_gpu_drivers.py tests/test_gpu_fullsize.py -k "ilu or config3 or drivers" -q -x -rf \
    --timeout 300 --timeout-method thread > "$O/pytest.log" 2>&1
rc=$?; tail -3 "$O/pytest.log"; [ $rc -eq 0 ] || exit $rc
for r in $(seq 1 "${ROUNDS:-1}"); do
    for v in r3 0 1; do
        if [ $v = r3 ]; then P=$PWD/respasol_amd/build/ab/r3/librsp.so; M=0; else P=""; M=$v; fi
        RSP_PROBE_LIB=$P RSP_ILU_FLOW_MODE=$M timeout -k 10 600 python scripts/bench_ilu0.py --reps 3 > "$O/${v}_$r.txt" 2> "$O/${v}_$r.err" \
            || { tail -20 "$O/${v}_$r.err"; exit 1; }
        echo "$v round $r: $(tail -1 "$O/${v}_$r.txt")"
    done
done
