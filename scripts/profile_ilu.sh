#!/bin/bash
# rocprofv3 kernel trace of the config-3 ILU(0) run + the config-1 CPU SpMV
# (reference methodology: one cold call, 4 pinned threads; and all threads).
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
TAG=${1:-ilu}
OUT="$ROOT/gpurun_out/$TAG"
mkdir -p "$OUT"
export TMPDIR=/tmp
cd /tmp
cd "$ROOT"
timeout -k 10 300 python3 scripts/bench_ilu0.py --json "$OUT/ilu.json" > "$OUT/ilu.out" 2> "$OUT/ilu.err"
rc=$?; echo "ilu rc=$rc"; [ $rc -ne 0 ] && exit $rc
cd /tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/ilustats" -o run -- \
    python3 "$ROOT/scripts/bench_ilu0.py" --reps 3 > "$OUT/ilu_prof.txt" 2> "$OUT/ilu_prof.err"
rc=$?; echo "ilu stats rc=$rc"; [ $rc -ne 0 ] && exit $rc
cd "$ROOT"
lscpu | grep -E "Model name|Socket|Core|Thread|^CPU\(s\)" > "$OUT/lscpu.txt"
for t in 4 16; do
  for rep in 1 2 3; do
    OMP_NUM_THREADS=$t OMP_PROC_BIND=close timeout -k 10 120 respasol_amd/bin/test_spmv_cpu \
        surrogate:2cubes_sphere "$OUT/config1_t$t.csv" || exit 1
  done
done
cat "$OUT/lscpu.txt" "$OUT"/config1_t*.csv
