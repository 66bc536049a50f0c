#!/bin/bash
# One GPU session on the box: smoke -> GPU tests -> bench -> rocprofv3 stats.
# Every GPU step has its own time limit; a fault / abort / segfault / timeout
# (exit >= 124 or >= 128) ends the script at once. Ordinary test failures
# (pytest exit 1) are recorded and the session continues.
# Usage: scripts/gpu_check.sh [tag] [steps]
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=${1:-r01}
STEPS=${2:-20}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp

fatal() { # rc step
    if [ "$1" -ge 124 ]; then echo "STOP: $2 exited $1 (fault/timeout)"; exit "$1"; fi
}

echo "== smoke"; timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1
rc=$?; echo "smoke rc=$rc"; tail -3 "$OUT/smoke.log"; fatal $rc smoke
[ $rc -ne 0 ] && exit $rc

echo "== pytest -m gpu"; timeout -k 10 900 python -m pytest tests -m gpu -q -rf > "$OUT/pytest_gpu.log" 2>&1
rc=$?; echo "pytest rc=$rc"; tail -15 "$OUT/pytest_gpu.log"; fatal $rc pytest

echo "== bench"; timeout -k 10 600 python bench.py --steps "$STEPS" --warmup 3 > "$OUT/bench.json" 2> "$OUT/bench.err"
rc=$?; echo "bench rc=$rc"; cat "$OUT/bench.json"; tail -5 "$OUT/bench.err"; fatal $rc bench

echo "== rocprofv3 kernel stats"
cd /tmp && timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$GRAFT_REPO_ROOT/$OUT/prof" -o run -- \
    python3 "$GRAFT_REPO_ROOT/bench.py" --steps "$STEPS" --warmup 3 --no-cpu > "$GRAFT_REPO_ROOT/$OUT/bench_prof.json" 2> "$GRAFT_REPO_ROOT/$OUT/prof.err"
rc=$?; cd "$GRAFT_REPO_ROOT"; echo "rocprof rc=$rc"; fatal $rc rocprof
find "$OUT/prof" -name "*kernel_stats*" | head -3
exit 0
