#!/bin/bash
# Same-box A/B of this tree against a git worktree of an earlier commit at
# ab_old/ (built in place): fp64 config 3, interleaved, 2 passes.
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
TAG=$1; shift
OUT="$ROOT/gpurun_out/$TAG"
mkdir -p "$OUT"
export TMPDIR=/tmp
for pass in 1 2; do
  for side in new old; do
    dir="$ROOT"; [ $side = old ] && dir="$ROOT/ab_old"
    (cd "$dir" && env "$@" timeout -k 10 200 python scripts/bench_ilu0.py --fp64-only --reps 3) \
        > "$OUT/$side.p$pass.txt" 2> "$OUT/$side.p$pass.err" || { echo "FAIL $side"; tail -5 "$OUT/$side.p$pass.err"; exit 1; }
    echo "[$side] pass $pass: $(grep '^TOTAL' "$OUT/$side.p$pass.txt" | cut -d';' -f1)"
  done
done
