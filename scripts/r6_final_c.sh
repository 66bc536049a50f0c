#!/bin/bash
# Round 6 session C: the full GPU suite, the config-3 ILU bench, the analysis phase timing.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/${1:-r06d}
bash scripts/r6_final_a.sh ${1:-r06d} || exit 1
grep ANALYSIS "$O/ilu_config3.txt"
RSP_ILU_TIMING=1 timeout -k 10 300 python scripts/ilu_analysis_timing.py moderate 2 > "$O/an_timing.txt" 2>&1 || exit 1
tail -1 "$O/an_timing.txt"
