#!/bin/bash
# Profiling session (tag argument): the headline roofline evidence (fp64 + fp32),
# the moderate-set HBM traffic and the random-band counters.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$PWD
export TMPDIR=/tmp
T=${1:-r05}
[ "${SKIP_ROUND:-0}" = 1 ] || bash scripts/profile_round.sh $T || exit 1
O=$ROOT/gpurun_out/${T}m
mkdir -p "$O"
cd /tmp
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$O/fetch" -o run -- \
    python3 "$ROOT/scripts/pmc_run.py" --set moderate --meta "$O/meta.json" > "$O/fetch.log" 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$O/write" -o run -- \
    python3 "$ROOT/scripts/pmc_run.py" --set moderate > "$O/write.log" 2>&1 || exit 1
cd "$ROOT"
python3 scripts/pmc_summary.py --fetch "$O/fetch" --write "$O/write" --meta "$O/meta.json" --workload moderate \
    --out "$O/${T}m_pmc.json" || exit 1
python3 scripts/pmc_summary.py --fetch "$O/fetch" --write "$O/write" --meta "$O/meta.json" --workload moderate \
    --dtype f32 --out "$O/${T}m_pmc_f32.json" || exit 1
PMC_RUN_ARGS="--set cage13,Si87H76,Serena,Hook_1498" bash scripts/pmc_probe.sh ${T}rb || exit 1
python3 scripts/pmc_probe.py gpurun_out/${T}rb/p* --by-grid --kernels "spmv_tiles<double,spmv_tiles<float" \
    --out gpurun_out/${T}rb/probe_by_matrix.json > /dev/null
bash scripts/pmc_probe.sh ${T}probe || exit 1
echo done
