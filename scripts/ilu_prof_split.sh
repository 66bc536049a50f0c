#!/bin/bash
# Where config-3 factor / solve time goes on the box (diagnostics): per-chunk
# factor stamps (RSP_ILU_FTRACE) and a rocprofv3 kernel trace of one fp64
# factor + solve per named matrix, summarised per matrix and kernel.
#   bash scripts/ilu_prof_split.sh <tag> m1,m2,...
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
TAG=$1; M=$2
OUT="$ROOT/gpurun_out/$TAG"
mkdir -p "$OUT"
export TMPDIR=/tmp
cd "$ROOT"
timeout -k 10 300 python scripts/ilu_ftrace.py "$M" > "$OUT/ftrace.txt" 2>&1
rc=$?; echo "ftrace rc=$rc"; grep -v amdgpu "$OUT/ftrace.txt"; [ $rc -ne 0 ] && exit $rc
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d "$OUT/kt" -o run -- \
    python3 "$ROOT/scripts/bench_ilu0.py" --set "$M" --fp64-only --reps 1 > "$OUT/bench.txt" 2> "$OUT/bench.err"
rc=$?; echo "trace rc=$rc"; [ $rc -ne 0 ] && exit $rc
cd "$ROOT"
python3 scripts/ilu_trace_split.py "$OUT/kt" "$M" > "$OUT/split.txt" 2>&1; cat "$OUT/split.txt"
