# round-5 GPU session: full suite, the PF narrow loops' parity, ILU A/B on the deep set
set -o pipefail
O=gpurun_out/${TAG:-r5b}
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1; rc=$?
echo "suite rc=$rc"; tail -3 $O/pytest.log
[ $rc -eq 0 ] || exit $rc
for pf in 1 2; do
RSP_ILU_NARROW_PF=$pf timeout -k 10 400 python -u -m pytest tests/test_gpu_ilu0.py tests/test_gpu_fullsize.py -k "ilu or trsv or solve" -x -q --timeout 300 --timeout-method thread > $O/pytest_pf$pf.log 2>&1; rc=$?
echo "pf$pf rc=$rc"; tail -3 $O/pytest_pf$pf.log
[ $rc -eq 0 ] || exit $rc
done
SET=dc1,G2_circuit,matrix-new_3,thermomech_TK ROUNDS=2 timeout -k 10 500 bash scripts/env_ab.sh ${TAG:-r5b}/ab "base:RSP_ILU_NARROW_PF=0" "pf1:RSP_ILU_NARROW_PF=1" "pf2:RSP_ILU_NARROW_PF=2"
