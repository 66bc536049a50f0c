#!/bin/bash
# Per-call floor: kernel duration vs inter-dispatch gap of back-to-back calls.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$PWD
O=$ROOT/gpurun_out/${1:-percall}
mkdir -p "$O"
export TMPDIR=/tmp
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d "$O/kt" -o run -- \
    python3 "$ROOT/scripts/spmv_ab.py" --set moderate --mode hot --variants 0 --rounds 1 > "$O/hot.txt" 2>&1
rc=$?; tail -3 "$O/hot.txt"; [ $rc -eq 0 ] || exit $rc
cd "$ROOT"
python3 scripts/percall_trace.py "$O/kt" > "$O/percall.txt"; cat "$O/percall.txt"
