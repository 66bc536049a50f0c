#!/bin/bash
# Full GPU validation pass: GPU tests, bench (big + moderate), ILU config 3,
# rocprofv3 profile. Each GPU step has its own time limit; stop at the first
# failure.
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
TAG=${1:-check}
OUT="$ROOT/gpurun_out/$TAG"
mkdir -p "$OUT"
cd "$ROOT"
step() {  # name, limit, command...
    local name=$1 lim=$2; shift 2
    echo "== $name"
    timeout -k 10 "$lim" "$@" > "$OUT/$name.out" 2> "$OUT/$name.err"
    local rc=$?
    echo "$name rc=$rc"; tail -3 "$OUT/$name.out"
    if [ $rc -ne 0 ]; then tail -20 "$OUT/$name.err"; exit $rc; fi
}
step pytest_gpu 900 python -m pytest tests -m gpu -q -rf -x
step bench 600 python bench.py
step bench_moderate 600 python bench.py --workload moderate --no-cpu
step ilu 600 python scripts/bench_ilu0.py --json "$OUT/ilu.json"
bash scripts/profile.sh "$TAG"
