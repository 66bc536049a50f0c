#!/bin/bash
# Round 4: deep-level solve A/B — the 4-wave narrow runs in the reference's
# term order (default), the one-wave narrow runs (RSP_ILU_NARROW_SPLIT=1, G
# by the plan / 2), the split term order (RSP_ILU_SPLIT=1), the round-3 library.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/${1:-r4split}
mkdir -p "$O"
export TMPDIR=/tmp
SET=${SET:-dc1,G2_circuit,matrix-new_3,thermomech_TK,ecology2,parabolic_fem,crashbasis,Dubcova3}
if [ "${PYTEST:-1}" = 1 ]; then
    timeout -k 10 600 python -u -m pytest tests/test_gpu_ilu0.py -q -x -rf --timeout 300 --timeout-method thread > "$O/pytest.log" 2>&1
    rc=$?; tail -3 "$O/pytest.log"; [ $rc -eq 0 ] || exit $rc
fi
for r in $(seq 1 "${ROUNDS:-2}"); do
    for v in ${VARIANTS:-def ns1 ns1g2 split r3}; do
        P=""; E="RSP_ILU_SPLIT=0"
        case $v in
            ns1) E="RSP_ILU_NARROW_SPLIT=1" ;;
            ns1g2) E="RSP_ILU_NARROW_SPLIT=1 RSP_ILU_GROUP=2" ;;
            split) E="RSP_ILU_SPLIT=1 RSP_ILU_NARROW_SPLIT=1" ;;
            r3) P=$PWD/respasol_amd/build/ab/r3/librsp.so ;;
            p_*) P=$PWD/respasol_amd/build/probe/${v#p_}/librsp.so ;;  # a probe build (make probe)
        esac
        env $E RSP_PROBE_LIB=$P timeout -k 10 300 python scripts/bench_ilu0.py --set "$SET" --fp64-only --reps 5 \
            > "$O/${v}_$r.txt" 2> "$O/${v}_$r.err" || { tail -20 "$O/${v}_$r.err"; exit 1; }
        echo "$v round $r: $(tail -1 "$O/${v}_$r.txt")"
    done
done
