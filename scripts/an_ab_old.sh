#!/bin/bash
# Same-box A/B of the ILU analysis wall time (config 3) against the ab_old
# worktree: interleaved, 3 passes; prints each side's total.
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
TAG=$1
OUT="$ROOT/gpurun_out/$TAG"
mkdir -p "$OUT"
M=2cubes_sphere,ASIC_320ks,Baumann,cfd2,crashbasis,ct20stif,dc1,Dubcova3,ecology2,FEM_3D_thermal2,G2_circuit,Goodwin_095,matrix-new_3,offshore,para-10,parabolic_fem,ss1,stomach,thermomech_TK,tmt_unsym,xenon2
for pass in 1 2 3; do
  for side in new old; do
    dir="$ROOT"; [ $side = old ] && dir="$ROOT/ab_old"
    (cd "$dir" && RSP_ILU_TIMING=1 timeout -k 10 200 python scripts/ilu_analysis_timing.py $M) \
        > "$OUT/$side.p$pass.txt" 2>&1 || { echo "FAIL $side"; tail -5 "$OUT/$side.p$pass.txt"; exit 1; }
    echo "[$side] pass $pass: $(grep ': analysis' "$OUT/$side.p$pass.txt" | awk '{s += $3} END {print s}') ms"
  done
done
