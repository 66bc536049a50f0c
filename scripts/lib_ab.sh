#!/bin/bash
# Interleaved A/B of two librsp.so builds on the ILU bench (diagnostics):
#   SET=a,b,c LIBS="respasol_amd/build/ab/old/librsp.so respasol_amd/lib/librsp.so" bash scripts/lib_ab.sh <tag>
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=${1:-libab}
O=gpurun_out/$TAG
mkdir -p "$O"
for r in $(seq 1 "${ROUNDS:-2}"); do
  i=0
  for lib in ${LIBS}; do
    i=$((i + 1))
    RSP_PROBE_LIB=$PWD/$lib timeout -k 10 300 python scripts/bench_ilu0.py --set "${SET}" > "$O/l${i}_r$r.txt" 2>&1 || { tail -20 "$O/l${i}_r$r.txt"; exit 1; }
    echo "== lib $i ($lib) round $r"; grep -v "amdgpu.ids\|median" "$O/l${i}_r$r.txt" | awk '{print $1, $6, $7, $10, $11}'
  done
done
