#!/bin/bash
# Interleaved A/B of the narrow-run wave counts (RSP_ILU_NARROW_WAVES for the
# solves, RSP_ILU_FNARROW_WAVES for the factor) on the ILU bench (diagnostics).
#   SET=dc1,G2_circuit WAVES="2 3 4 6 8" ROUNDS=2 bash scripts/waves_ab.sh <tag>
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=${1:-wavesab}
O=gpurun_out/$TAG
mkdir -p "$O"
for r in $(seq 1 "${ROUNDS:-2}"); do
  for w in ${WAVES}; do
    RSP_ILU_NARROW_WAVES=$w RSP_ILU_FNARROW_WAVES=$w timeout -k 10 300 python scripts/bench_ilu0.py --set "${SET}" --fp64-only > "$O/w${w}_r$r.txt" 2>&1 || { tail -20 "$O/w${w}_r$r.txt"; exit 1; }
    echo "== waves $w round $r: $(tail -1 "$O/w${w}_r$r.txt")"
  done
done
