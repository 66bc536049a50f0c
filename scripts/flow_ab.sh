#!/bin/bash
# A/B of the flow-segment solve knobs on the box (same process order twice).
# usage: scripts/flow_ab.sh OUTDIR SET "FLOW:WPC:SLEEP:GATE ..."
set -o pipefail
OUT=$1; SET=$2; CONFS=$3
mkdir -p "$OUT"
for pass in 1 2; do
  for c in $CONFS; do
    IFS=: read F W S G <<< "$c"
    RSP_ILU_FLOW=$F RSP_ILU_FLOW_WPC=$W RSP_ILU_FLOW_SLEEP=$S RSP_ILU_FLOW_GATE=${G:-1} timeout -k 10 200 \
      python scripts/bench_ilu0.py --set "$SET" > "$OUT/$c.$pass.txt" 2>&1 || exit 1
    echo "== $c pass $pass: $(grep '^TOTAL' "$OUT/$c.$pass.txt")"
  done
done
