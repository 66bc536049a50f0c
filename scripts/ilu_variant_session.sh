# ILU variant session: parity of each VARIANTS env setting, then an env A/B (ARMS) on the deep set
set -o pipefail
O=gpurun_out/${TAG:-ilu_var}
mkdir -p $O
for v in ${VARIANTS:-"RSP_ILU_LOADERS=1"}; do
env ${v//,/ } timeout -k 10 400 python -u -m pytest tests/test_gpu_ilu0.py tests/test_gpu_fullsize.py -k "ilu or trsv or solve" -x -q --timeout 300 --timeout-method thread > $O/pytest_$v.log 2>&1; rc=$?
echo "$v rc=$rc"; tail -2 $O/pytest_$v.log
[ $rc -eq 0 ] || exit $rc
done
SET=${SET:-dc1,G2_circuit,matrix-new_3,thermomech_TK} ROUNDS=${ROUNDS:-2} timeout -k 10 500 bash scripts/env_ab.sh ${TAG:-ilu_var}/ab ${ARMS:-"base:RSP_ILU_LOADERS=0" "ldr:RSP_ILU_LOADERS=1"}
