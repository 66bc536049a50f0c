#!/bin/bash
# Round-end evidence on one MI355X: every GPU test, config 3 (ILU) with a
# rocprofv3 kernel summary and the analysis phases, config 2 and the
# driver's own bench command (config 4 + config 5 Serena step).
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
TAG=${1:-final}
OUT="$ROOT/gpurun_out/$TAG"
mkdir -p "$OUT"
cd "$ROOT"
export TMPDIR=/tmp
step() {  # name, limit, command...
    local name=$1 lim=$2; shift 2
    echo "== $name"
    timeout -k 10 "$lim" "$@" > "$OUT/$name.out" 2> "$OUT/$name.err"
    local rc=$?
    echo "$name rc=$rc"; tail -2 "$OUT/$name.out"
    if [ $rc -ne 0 ]; then tail -20 "$OUT/$name.err"; exit $rc; fi
}
M=2cubes_sphere,ASIC_320ks,Baumann,cfd2,crashbasis,ct20stif,dc1,Dubcova3,ecology2,FEM_3D_thermal2,G2_circuit,Goodwin_095,matrix-new_3,offshore,para-10,parabolic_fem,ss1,stomach,thermomech_TK,tmt_unsym,xenon2
step pytest_gpu 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread
step ilu 300 python scripts/bench_ilu0.py --json "$OUT/ilu.json"
RSP_ILU_TIMING=1 step an_timing 300 python scripts/ilu_analysis_timing.py $M
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/ilustats" -o run -- \
    python3 "$ROOT/scripts/bench_ilu0.py" --fp64-only --reps 3 > "$OUT/ilu_prof.txt" 2> "$OUT/ilu_prof.err"
rc=$?; echo "ilu stats rc=$rc"; [ $rc -ne 0 ] && exit $rc
cd "$ROOT"
step bench_moderate 300 python bench.py --workload moderate --no-cpu
step bench 300 python bench.py --gpus 1 --steps 20 --warmup 5
