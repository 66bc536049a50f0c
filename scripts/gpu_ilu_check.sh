#!/bin/bash
# ILU GPU tests + config-3 ILU bench + analysis phase timing; each step
# time-limited, stop at the first failure. Usage: scripts/gpu_ilu_check.sh <tag>
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
TAG=${1:-ilucheck}
OUT="$ROOT/gpurun_out/$TAG"
mkdir -p "$OUT"
cd "$ROOT"
timeout -k 10 600 python -u -m pytest tests/test_gpu_ilu0.py tests/test_gpu_fullsize.py -m gpu -x -q --timeout 120 --timeout-method thread -k "ilu or analysis or Ilu" > "$OUT/pytest_ilu.log" 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 "$OUT/pytest_ilu.log"; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u scripts/ilu_analysis_timing.py moderate 3 > "$OUT/timing.txt" 2>&1
rc=$?; echo "timing rc=$rc"; grep total "$OUT/timing.txt"; [ $rc -ne 0 ] && exit $rc
if [ "${2:-}" = "bench" ]; then
  timeout -k 10 600 python -u scripts/bench_ilu0.py --json "$OUT/ilu.json" > "$OUT/ilu.txt" 2>&1
  rc=$?; echo "ilu rc=$rc"; tail -2 "$OUT/ilu.txt"; [ $rc -ne 0 ] && exit $rc
fi
exit 0
