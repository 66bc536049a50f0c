# round 6: factor-plan piece size (RSP_ILU_PIECE_ITEMS fixed) vs the adaptive default
# (1/32 of the thin positions within [2^15, 2^16]): analysis phase sums (moderate,
# 2 calls) and the circuits' fp64 factor / solve, interleaved on one box
set -u
O=gpurun_out/${TAG:-r6piece}
mkdir -p $O
SET=${SET:-dc1,matrix-new_3,ASIC_320ks,ss1,xenon2,G2_circuit,thermomech_TK,crashbasis}
for arm in ${ARMS:-cur p16k:RSP_ILU_PIECE_ITEMS=16384 p8k:RSP_ILU_PIECE_ITEMS=8192 cur2 p16kb:RSP_ILU_PIECE_ITEMS=16384 p8kb:RSP_ILU_PIECE_ITEMS=8192}; do
  name=${arm%%:*}; envs=${arm#*:}; [ "$envs" = "$arm" ] && envs=""
  env $envs RSP_ILU_TIMING=1 timeout -k 10 300 python scripts/ilu_analysis_timing.py moderate 2 > $O/${name}_an.txt 2>&1 || exit 1
  env $envs timeout -k 10 300 python scripts/bench_ilu0.py --set $SET --fp64-only --reps 5 > $O/${name}.txt 2>&1 || exit 1
  echo "$name: an $(tail -1 $O/${name}_an.txt) | $(grep TOTAL $O/${name}.txt | cut -c1-45)"
done
