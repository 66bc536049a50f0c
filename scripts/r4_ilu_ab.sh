#!/bin/bash
# Round 4: ILU GPU tests, then config-3 timing of the round-3 library
# (respasol_amd/build/ab/r3/librsp.so, static flow items, relaxed flag
# hand-off) against the current one (claimed flow items, release/acquire).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=${1:-r4ilu}
O=gpurun_out/$TAG
mkdir -p "$O"
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_gpu_ilu0.py tests/test_gpu_drivers.py -q -x -rf \
    --timeout 300 --timeout-method thread > "$O/pytest.log" 2>&1
rc=$?; tail -3 "$O/pytest.log"; [ $rc -eq 0 ] || exit $rc
for r in $(seq 1 "${ROUNDS:-2}"); do
    for lib in r3 cur; do
        if [ $lib = r3 ]; then P=$PWD/respasol_amd/build/ab/r3/librsp.so; else P=""; fi
        RSP_PROBE_LIB=$P timeout -k 10 600 python scripts/bench_ilu0.py --reps 3 > "$O/${lib}_$r.txt" 2> "$O/${lib}_$r.err" \
            || { tail -20 "$O/${lib}_$r.err"; exit 1; }
        echo "$lib round $r: $(tail -1 "$O/${lib}_$r.txt")"
    done
done
