#!/bin/bash
# GPU tests + (optional) ILU config-3 bench; each step time-limited, stop on failure.
# Usage: scripts/quick_gpu.sh <tag> [ilu]
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
TAG=${1:-quick}
OUT="$ROOT/gpurun_out/$TAG"
mkdir -p "$OUT"
cd "$ROOT"
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > "$OUT/pytest_gpu.log" 2>&1
rc=$?; echo "pytest rc=$rc"; tail -5 "$OUT/pytest_gpu.log"; [ $rc -ne 0 ] && exit $rc
if [ "${2:-}" = "ilu" ]; then
  timeout -k 10 600 python -u scripts/bench_ilu0.py --json "$OUT/ilu.json" > "$OUT/ilu.txt" 2>&1
  rc=$?; echo "ilu rc=$rc"; tail -4 "$OUT/ilu.txt"; [ $rc -ne 0 ] && exit $rc
fi
exit 0
