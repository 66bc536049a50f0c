#!/bin/bash
# PMC passes (one counter group per run) over the ILU solves of one surrogate.
#   bash scripts/ilu_pmc.sh <tag> <matrix>
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
TAG=${1:-ilupmc}; M=${2:-ecology2}
OUT="$ROOT/gpurun_out/$TAG"
mkdir -p "$OUT"
export TMPDIR=/tmp
cd /tmp
i=0
for grp in ${GROUPS_OVERRIDE:-"SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU" \
           "SQ_INSTS_LDS SQ_INSTS_VALU SQ_INSTS_SALU SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_INSTS_SMEM SQ_ACTIVE_INST_SCA SQ_INST_CYCLES_SALU"}; do
    i=$((i+1))
    timeout -s KILL 90 rocprofv3 --pmc $grp --output-format csv -d "$OUT/p$i" -o run -- python3 "$ROOT/scripts/ilu_pmc_run.py" "$M" > "$OUT/p$i.log" 2>&1
    rc=$?; echo "pass $i rc=$rc"; [ $rc -ne 0 ] && { tail -5 "$OUT/p$i.log"; exit $rc; }
done
exit 0
