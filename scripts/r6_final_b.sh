#!/bin/bash
# Round 6 session B (one box): the driver's bench command, then the same
# command under rocprofv3 --kernel-trace --stats with the PMC passes
# (profile_round.sh), then the config-2 bench — so profiles/ and the line
# come from the same session.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
T=${1:-r06}
O=gpurun_out/${T}b
mkdir -p "$O"
export TMPDIR=/tmp
timeout -k 10 300 python bench.py > "$O/bench_default.json" 2> "$O/bench_default.err" || exit 1
bash scripts/profile_round.sh $T || exit 1
timeout -k 10 300 python bench.py --workload moderate --no-cpu > "$O/bench_moderate.json" 2> "$O/bench_moderate.err" || exit 1
echo done
