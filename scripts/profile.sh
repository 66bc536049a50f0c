#!/bin/bash
# Profiling session on the GPU box (results copied to profiles/ by hand):
#   1. rocprofv3 --kernel-trace --stats on bench.py (kernel durations)
#   2. rocprofv3 --pmc FETCH_SIZE  on scripts/pmc_run.py  (own run)
#   3. rocprofv3 --pmc WRITE_SIZE  on scripts/pmc_run.py  (own run)
#   4. scripts/pmc_summary.py -> gpurun_out/<tag>/<tag>_pmc.json
# Each GPU step has its own time limit; stop at the first fault/timeout.
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
TAG=${1:-r01}
OUT="$ROOT/gpurun_out/$TAG"
mkdir -p "$OUT"
export TMPDIR=/tmp
cd /tmp
fatal() { if [ "$1" -ge 124 ]; then echo "STOP: $2 exited $1"; exit "$1"; fi; }
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/stats" -o run -- \
    python3 "$ROOT/bench.py" --steps 20 --warmup 3 --no-cpu > "$OUT/bench_prof.json" 2> "$OUT/stats.err"
rc=$?; echo "stats rc=$rc"; fatal $rc stats
timeout -k 10 600 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$OUT/fetch" -o run -- \
    python3 "$ROOT/scripts/pmc_run.py" --meta "$OUT/meta.json" > "$OUT/fetch.log" 2>&1
rc=$?; echo "fetch rc=$rc"; fatal $rc fetch
timeout -k 10 600 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$OUT/write" -o run -- \
    python3 "$ROOT/scripts/pmc_run.py" > "$OUT/write.log" 2>&1
rc=$?; echo "write rc=$rc"; fatal $rc write
cd "$ROOT"
python3 scripts/pmc_summary.py --fetch "$OUT/fetch" --write "$OUT/write" --meta "$OUT/meta.json" \
    --out "$OUT/${TAG}_pmc.json"
