#!/bin/bash
# Round 4 GPU call: ILU parity (split solve order) + config-3 timing, then the
# SpMV counter probe. Each step under its own limit; stop at the first failure.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/${1:-r4f}
mkdir -p "$O"
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_ilu0.py tests/test_gpu_drivers.py tests/test_gpu_spmv_batch.py -q -x -rf \
    --timeout 300 --timeout-method thread > "$O/pytest.log" 2>&1
rc=$?; tail -3 "$O/pytest.log"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python scripts/bench_ilu0.py --reps 3 > "$O/ilu_config3.txt" 2> "$O/ilu_config3.err"
rc=$?; tail -1 "$O/ilu_config3.txt"; [ $rc -eq 0 ] || exit $rc
bash scripts/pmc_probe.sh ${1:-r4f}/probe
