#!/bin/bash
# Interleaved A/B of ILU knob settings on the box (fp64 config 3, 2 passes):
#   bash scripts/ilu_knob_ab.sh <tag> "A=1,B=2" "A=0" ...   ("-" = defaults)
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
TAG=$1; shift
OUT="$ROOT/gpurun_out/$TAG"
mkdir -p "$OUT"
cd "$ROOT"
export TMPDIR=/tmp
for pass in 1 2; do
  i=0
  for conf in "$@"; do
    i=$((i + 1))
    envs=()
    [ "$conf" != "-" ] && IFS=, read -ra envs <<< "$conf"
    env "${envs[@]}" timeout -k 10 200 python scripts/bench_ilu0.py --fp64-only --reps 3 \
        > "$OUT/c$i.p$pass.txt" 2> "$OUT/c$i.p$pass.err" || { echo "FAIL $conf"; tail -5 "$OUT/c$i.p$pass.err"; exit 1; }
    echo "[$conf] pass $pass: $(grep '^TOTAL' "$OUT/c$i.p$pass.txt" | cut -d';' -f1)"
  done
done
