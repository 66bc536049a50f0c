#!/bin/bash
# ILU GPU tests + one config-3 timing run (+ optional trace of named matrices).
#   bash scripts/ilu_check.sh <tag> [trace-matrices]
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=${1:-ilu}
O=gpurun_out/$TAG
mkdir -p "$O"
export TMPDIR=/tmp
timeout -k 10 600 python -m pytest tests/test_gpu_ilu0.py tests/test_gpu_drivers.py -q -x -rf > "$O/pytest.log" 2>&1
rc=$?; tail -3 "$O/pytest.log"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python scripts/bench_ilu0.py --json "$O/ilu.json" > "$O/ilu.txt" 2> "$O/ilu.err" || { tail -20 "$O/ilu.err"; exit 1; }
cat "$O/ilu.txt"
if [ -n "${2:-}" ]; then
    timeout -k 10 300 python scripts/ilu_trace.py "$2" > "$O/trace.txt" 2>&1 && \
    RSP_ILU_TRACE_CLK=1 timeout -k 10 300 python scripts/ilu_trace.py "$2" >> "$O/trace.txt" 2>&1
    grep -v amdgpu.ids "$O/trace.txt"
fi
