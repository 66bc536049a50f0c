#!/bin/bash
# ILU GPU tests + config-3 timing A/B of an environment knob:
#   KNOB=RSP_ILU_GROUP VALUES="2 4" bash scripts/ilu_ab.sh <tag>
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=${1:-iluab}
O=gpurun_out/$TAG
mkdir -p "$O"
export TMPDIR=/tmp
timeout -k 10 900 python -m pytest tests/test_gpu_ilu0.py tests/test_gpu_drivers.py -q -x -rf > "$O/pytest.log" 2>&1
rc=$?; tail -3 "$O/pytest.log"; [ $rc -eq 0 ] || exit $rc
for r in $(seq 1 "${ROUNDS:-1}"); do for v in ${VALUES:-0 1}; do
    env "${KNOB:-RSP_ILU_GROUP}=$v" timeout -k 10 600 python scripts/bench_ilu0.py > "$O/${v}_$r.txt" 2> "$O/${v}_$r.err" \
        || { tail -20 "$O/${v}_$r.err"; exit 1; }
    echo "${KNOB:-RSP_ILU_GROUP}=$v round $r: $(tail -1 "$O/${v}_$r.txt")"
done; done
