#!/bin/bash
# A/B of RSP_SPMV_VARIANT values on the bench (big set, N = 1), interleaved
# rounds: VARIANTS="0 32" ROUNDS=2 bash scripts/variant_ab.sh <tag> [bench args]
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=${1:-vab}; shift || true
O=gpurun_out/$TAG
mkdir -p "$O"
export TMPDIR=/tmp
[ -n "${TESTS:-}" ] && { timeout -k 10 900 python -m pytest $TESTS -q -x -rf > "$O/pytest.log" 2>&1;
    rc=$?; tail -5 "$O/pytest.log"; [ $rc -eq 0 ] || exit $rc; }
for r in $(seq 1 "${ROUNDS:-2}"); do for v in ${VARIANTS:-0 32}; do
    RSP_SPMV_VARIANT=$v timeout -k 10 300 python bench.py --steps 30 --warmup 3 --no-cpu "$@" \
        > "$O/v${v}_$r.json" 2> "$O/v${v}_$r.err" || { tail -20 "$O/v${v}_$r.err"; exit 1; }
    python - "$O/v${v}_$r.json" "v$v r$r" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).readlines()[-1])
print(sys.argv[2], "ms/step", d["ms_per_step"], "frac", d["roofline"]["frac"], "per-matrix ms",
      d["per_matrix_calls"]["ms_per_step_rank0"], "fp32 ms", d["fp32"]["ms_per_pass_rank0"], d["parity_check"])
PY
done; done
