#!/bin/bash
# End-of-round validation: GPU tests, smoke, the driver's bench command, the
# moderate bench, the config-3 ILU bench and the analysis timing. Each step
# time-limited; stop at the first failure. Usage: scripts/final_round3.sh <tag>
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
TAG=${1:-final}
OUT="$ROOT/gpurun_out/$TAG"
mkdir -p "$OUT"
cd "$ROOT"
step() {  # name, limit, command...
    local name=$1 lim=$2; shift 2
    timeout -k 10 "$lim" "$@" > "$OUT/$name.out" 2> "$OUT/$name.err"
    local rc=$?
    echo "$name rc=$rc: $(tail -1 "$OUT/$name.out" | cut -c1-200)"
    if [ $rc -ne 0 ]; then tail -20 "$OUT/$name.err"; exit $rc; fi
}
step pytest_gpu 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread
step smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
step bench 300 python bench.py --gpus 1 --steps 20 --warmup 5
step bench_moderate 300 python bench.py --workload moderate --no-cpu
step ilu 600 python -u scripts/bench_ilu0.py --json "$OUT/ilu.json"
step an_timing 300 python -u scripts/ilu_analysis_timing.py moderate 3
exit 0
