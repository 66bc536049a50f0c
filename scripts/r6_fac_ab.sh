# round 6: narrow factor runs, third round prefetched (current) vs two (probe), interleaved
set -u
O=gpurun_out/${TAG:-r6fac}
mkdir -p $O
P=$PWD/respasol_amd/build/probe
SET=${SET:-dc1,matrix-new_3,thermomech_TK,ASIC_320ks,ss1,tmt_unsym}
for arm in ${ARMS:-cur "pre2:RSP_PROBE_LIB=$P/pre2/librsp.so" cur2 "pre2b:RSP_PROBE_LIB=$P/pre2/librsp.so"}; do
  name=${arm%%:*}; envs=${arm#*:}; [ "$envs" = "$arm" ] && envs=""
  env $envs timeout -k 10 300 python scripts/bench_ilu0.py --set $SET --reps 5 > $O/${name}.txt 2>&1 || exit 1
  echo "$name: $(grep TOTAL $O/${name}.txt)"
  grep -E "^(dc1|matrix-new_3) " $O/${name}.txt | cut -c1-110
done
