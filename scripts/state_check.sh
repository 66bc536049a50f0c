#!/bin/bash
# One GPU pass over the current tree: GPU tests, config-3 ILU timing, bench.
# Each GPU step has its own limit; the script stops at the first failure.
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
TAG=${1:-state}
OUT="$ROOT/gpurun_out/$TAG"
mkdir -p "$OUT"
cd "$ROOT"
export TMPDIR=/tmp
step() {  # name, limit, command...
    local name=$1 lim=$2; shift 2
    echo "== $name"
    timeout -k 10 "$lim" "$@" > "$OUT/$name.out" 2> "$OUT/$name.err"
    local rc=$?
    echo "$name rc=$rc"; tail -3 "$OUT/$name.out"
    if [ $rc -ne 0 ]; then tail -20 "$OUT/$name.err"; exit $rc; fi
}
[ "${SKIP_TESTS:-0}" = 1 ] || step pytest_gpu 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread
step ilu 300 python scripts/bench_ilu0.py --json "$OUT/ilu.json"
[ "${SKIP_BENCH:-0}" = 1 ] || step bench 300 python bench.py
