#!/bin/bash
# ILU pass on the GPU box: ILU GPU tests, analysis phase times
# (RSP_ILU_TIMING=2) over config 3, config-3 factor / solve timing.
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
TAG=${1:-ilu}
OUT="$ROOT/gpurun_out/$TAG"
mkdir -p "$OUT"
cd "$ROOT"
export TMPDIR=/tmp
step() {  # name, limit, command...
    local name=$1 lim=$2; shift 2
    echo "== $name"
    timeout -k 10 "$lim" "$@" > "$OUT/$name.out" 2> "$OUT/$name.err"
    local rc=$?
    echo "$name rc=$rc"; tail -3 "$OUT/$name.out"
    if [ $rc -ne 0 ]; then tail -20 "$OUT/$name.err"; exit $rc; fi
}
M=2cubes_sphere,ASIC_320ks,Baumann,cfd2,crashbasis,ct20stif,dc1,Dubcova3,ecology2,FEM_3D_thermal2,G2_circuit,Goodwin_095,matrix-new_3,offshore,para-10,parabolic_fem,ss1,stomach,thermomech_TK,tmt_unsym,xenon2
[ "${SKIP_TESTS:-0}" = 1 ] || step pytest_ilu 600 python -u -m pytest tests/test_gpu_ilu0.py tests/test_gpu_drivers.py -x -q --timeout 300 --timeout-method thread
RSP_ILU_TIMING=2 step an_timing 300 python scripts/ilu_analysis_timing.py $M
step ilu 300 python scripts/bench_ilu0.py --json "$OUT/ilu.json"
