#!/bin/bash
# Interleaved A/B of two librsp.so builds on bench.py (SpMV, diagnostics):
#   LIBS="respasol_amd/build/ab/old/librsp.so respasol_amd/lib/librsp.so" WORKLOAD=moderate bash scripts/lib_ab_spmv.sh <tag>
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=${1:-spmvab}
O=gpurun_out/$TAG
mkdir -p "$O"
for r in $(seq 1 "${ROUNDS:-2}"); do
  i=0
  for lib in ${LIBS}; do
    i=$((i + 1))
    RSP_PROBE_LIB=$PWD/$lib timeout -k 10 300 python bench.py --workload "${WORKLOAD:-moderate}" --no-cpu --steps 20 > "$O/l${i}_r$r.json" 2> "$O/l${i}_r$r.err" || { tail -20 "$O/l${i}_r$r.err"; exit 1; }
    python3 - "$O/l${i}_r$r.json" "$lib" "$r" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
pm = d["per_matrix_us_rank0"]
print(f"lib {sys.argv[2]} round {sys.argv[3]}: batched {d['value']} GFLOP/s frac {d['roofline']['frac']}; "
      f"per-call step {d['per_matrix_calls']['ms_per_step_rank0']} ms frac {d['per_matrix_calls']['frac_rank0']}; "
      + " ".join(f"{k}={v}" for k, v in pm.items() if k in ("ASIC_320ks", "ss1", "dc1", "matrix-new_3", "G2_circuit")))
PY
  done
done
