#!/bin/bash
# Interleaved A/B of two librsp.so builds on bench.py (diagnostics):
#   LIBS="respasol_amd/build/ab/old/librsp.so respasol_amd/lib/librsp.so" bash scripts/bench_lib_ab.sh <tag> [bench args]
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=${1:-blab}
shift || true
O=gpurun_out/$TAG
mkdir -p "$O"
for r in $(seq 1 "${ROUNDS:-2}"); do
  i=0
  for lib in ${LIBS}; do
    i=$((i + 1))
    RSP_PROBE_LIB=$PWD/$lib timeout -k 10 300 python bench.py --steps 30 --warmup 3 --no-cpu "$@" > "$O/l${i}_r$r.json" 2> "$O/l${i}_r$r.err" || { tail -20 "$O/l${i}_r$r.err"; exit 1; }
    python - "$O/l${i}_r$r.json" "$i" "$r" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print(f"lib{sys.argv[2]} r{sys.argv[3]} ms/step", d["ms_per_step"], "frac", d["roofline"]["frac"],
      "per-matrix ms", d["per_matrix_calls"]["ms_per_step_rank0"], "fp32 ms",
      d["fp32"]["ms_per_pass_rank0"], d["parity_check"])
PY
  done
done
