#!/bin/bash
# SpMV GPU tests with an RSP_SPMV_VARIANT set, then an interleaved bench A/B:
#   WV=64 VARIANTS="0 64" bash scripts/variant_test_ab.sh <tag> [bench args]
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=${1:-vtab}; shift || true
O=gpurun_out/$TAG
mkdir -p "$O"
RSP_SPMV_VARIANT=${WV:-0} timeout -k 10 600 python -u -m pytest tests/test_gpu_spmv.py tests/test_gpu_spmv_batch.py \
    -x -q --timeout 120 --timeout-method thread > "$O/pytest_variant.log" 2>&1
rc=$?; tail -2 "$O/pytest_variant.log"; [ $rc -eq 0 ] || exit $rc
VARIANTS="${VARIANTS:-0 64}" ROUNDS="${ROUNDS:-2}" bash scripts/variant_ab.sh "$TAG" "$@"
