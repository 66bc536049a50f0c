# round 6: block-inverse solve parity + deep-set timing, then the flow ticket A/B
set -o pipefail
O=gpurun_out/${TAG:-r6b2}
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_blocks.py -x -v --timeout 120 --timeout-method thread > $O/pytest_blocks.log 2>&1; rc=$?
tail -15 $O/pytest_blocks.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u scripts/bench_ilu0.py --set dc1,G2_circuit,matrix-new_3,thermomech_TK --reps 5 > $O/deep.txt 2>&1 || { tail -20 $O/deep.txt; exit 1; }
cat $O/deep.txt
RSP_ILU_BLOCKS=0 timeout -k 10 300 python -u scripts/bench_ilu0.py --set dc1,G2_circuit,matrix-new_3 --reps 5 --fp64-only > $O/deep_levels.txt 2>&1 || { tail -20 $O/deep_levels.txt; exit 1; }
cat $O/deep_levels.txt
if [ -n "$AB" ]; then
SET=moderate ROUNDS=2 timeout -k 10 900 bash scripts/env_ab.sh ${TAG:-r6b2}/ab "static:RSP_ILU_FLOW_MODE=0" "ticket:RSP_ILU_FLOW_MODE=2"
fi
