set -o pipefail
mkdir -p gpurun_out/${TAG:-r6a}
timeout -k 10 400 python -u -m pytest tests/test_gpu_ilu0.py -k "flow" -x -v --timeout 120 --timeout-method thread > gpurun_out/${TAG:-r6a}/pytest_flow.log 2>&1; rc=$?
tail -5 gpurun_out/${TAG:-r6a}/pytest_flow.log
[ $rc -eq 0 ] || exit $rc
SET=moderate ROUNDS=2 timeout -k 10 900 bash scripts/env_ab.sh ${TAG:-r6a}/ab "static:RSP_ILU_FLOW_MODE=0" "ticket:RSP_ILU_FLOW_MODE=2"
