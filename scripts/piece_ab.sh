#!/bin/bash
# A/B of the factor plan's piece size (RSP_ILU_PIECE_ITEMS): analysis time and
# config-3 factor/solve times. Usage: scripts/piece_ab.sh <tag> <items...>
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
TAG=$1; shift
OUT="$ROOT/gpurun_out/$TAG"
mkdir -p "$OUT"
cd "$ROOT"
for it in "$@"; do
  RSP_ILU_PIECE_ITEMS=$it timeout -k 10 300 python -u scripts/ilu_analysis_timing.py moderate 3 > "$OUT/timing_$it.txt" 2>&1
  rc=$?; echo "timing $it rc=$rc $(grep total "$OUT/timing_$it.txt")"; [ $rc -ne 0 ] && exit $rc
  RSP_ILU_PIECE_ITEMS=$it timeout -k 10 300 python -u scripts/bench_ilu0.py > "$OUT/ilu_$it.txt" 2>&1
  rc=$?; echo "ilu $it rc=$rc"; tail -1 "$OUT/ilu_$it.txt"; [ $rc -ne 0 ] && exit $rc
done
exit 0
