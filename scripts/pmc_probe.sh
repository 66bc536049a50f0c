#!/bin/bash
# Diagnostic counter passes over scripts/pmc_run.py (fp64 then fp32 big set):
# where the SpMV tile kernel's time goes (issue / wait split, TA / TD / TCP
# busy and stall cycles). One run per pass (slot limits: 8 SQ, 4 TCP, 2 TA,
# 2 TD, 2 GRBM), each under its own time limit; stop at the first failure.
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
TAG=${1:-probe}
OUT="$ROOT/gpurun_out/$TAG"
mkdir -p "$OUT"
export TMPDIR=/tmp
cd /tmp
P1="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_LDS SQ_INSTS_VMEM_RD SQ_BUSY_CYCLES GRBM_GUI_ACTIVE"
P2="TA_TA_BUSY TA_ADDR_STALLED_BY_TC_CYCLES TD_TD_BUSY TD_TC_STALL TCP_TOTAL_CACHE_ACCESSES TCP_TCP_TA_DATA_STALL_CYCLES TCP_TCC_READ_REQ TCP_PENDING_STALL_CYCLES GRBM_GUI_ACTIVE"
i=0
for P in "$P1" "$P2" ${EXTRA_PASSES:-}; do
    i=$((i + 1))
    timeout -s KILL 300 rocprofv3 --pmc $P --output-format csv -d "$OUT/p$i" -o run -- \
        python3 "$ROOT/scripts/pmc_run.py" --passes 3 ${PMC_RUN_ARGS:-} > "$OUT/p$i.log" 2>&1
    rc=$?; echo "pass $i rc=$rc"; if [ $rc -ne 0 ]; then tail -5 "$OUT/p$i.log"; exit $rc; fi
done
cd "$ROOT"
python3 scripts/pmc_probe.py "$OUT"/p* --out "$OUT/probe.json"
