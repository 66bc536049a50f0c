#!/bin/bash
# Round 6 session A: the full GPU suite and the config-3 ILU bench.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/${1:-r06a}
mkdir -p "$O"
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -rf --timeout 300 --timeout-method thread > "$O/pytest_gpu.txt" 2>&1
rc=$?; tail -3 "$O/pytest_gpu.txt"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python scripts/bench_ilu0.py --reps 3 --json "$O/ilu_config3.json" > "$O/ilu_config3.txt" 2> "$O/ilu_config3.err" || exit 1
tail -1 "$O/ilu_config3.txt"
