#!/bin/bash
# Round 4: SpMV gather lane-order probe (timing + TA counters), then the
# deep-level solve A/B (scripts/r4_split_ab.sh).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=${1:-r4c2}
O=gpurun_out/$TAG
mkdir -p "$O"
export TMPDIR=/tmp
timeout -k 10 400 python scripts/spmv_probe.py --probes base,emajor,loadsonly,nogather --rounds 2 > "$O/probe.txt" 2>&1
rc=$?; tail -12 "$O/probe.txt"; [ $rc -eq 0 ] || exit $rc
RSP_PROBE_LIB=$PWD/respasol_amd/build/probe/emajor/librsp.so bash scripts/pmc_probe.sh $TAG/pmc_emajor || exit 1
bash scripts/r4_split_ab.sh $TAG/split
