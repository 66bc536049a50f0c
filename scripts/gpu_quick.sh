#!/bin/bash
# Quick GPU iteration: GPU tests, bench, A/B of SpMV variants. Stops at the
# first fault/timeout (exit >= 124).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=${1:-quick}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
fatal() { if [ "$1" -ge 124 ]; then echo "STOP: $2 exited $1"; exit "$1"; fi; }
echo "== pytest -m gpu"; timeout -k 10 900 python -m pytest tests -m gpu -q -rf -x > "$OUT/pytest_gpu.log" 2>&1
rc=$?; echo "pytest rc=$rc"; tail -8 "$OUT/pytest_gpu.log"; fatal $rc pytest
echo "== bench"; timeout -k 10 600 python bench.py --steps 20 --warmup 3 --cpu-seconds 3 > "$OUT/bench.json" 2> "$OUT/bench.err"
rc=$?; echo "bench rc=$rc"; cat "$OUT/bench.json"; fatal $rc bench
echo "== A/B"; timeout -k 10 600 python scripts/spmv_ab.py ${AB_ARGS:-} > "$OUT/ab.txt" 2>&1
rc=$?; echo "ab rc=$rc"; cat "$OUT/ab.txt"; fatal $rc ab
