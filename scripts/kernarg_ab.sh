#!/bin/bash
# A/B: dependent-launch gap of the ILU fat levels with kernel arguments in
# device memory (HIP_FORCE_DEV_KERNARG=1) vs host memory (=0), interleaved.
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT="$ROOT/gpurun_out/${1:-kern}"
mkdir -p "$OUT"
cd "$ROOT"
for v in 0 1 0 1; do
  echo "== HIP_FORCE_DEV_KERNARG=$v"
  HIP_FORCE_DEV_KERNARG=$v timeout -k 10 300 python scripts/bench_ilu0.py --reps 3 > "$OUT/ilu_$v.txt" 2>&1 || exit 1
  tail -1 "$OUT/ilu_$v.txt"
done
