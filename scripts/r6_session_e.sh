# round 6: ticket fast-path diagnosis (probe builds)
set -u
O=gpurun_out/${TAG:-r6e}
mkdir -p $O
SET=${SET:-offshore,stomach,xenon2,para-10,2cubes_sphere,cfd2,FEM_3D_thermal2,Goodwin_095,tmt_unsym,ecology2,crashbasis,ASIC_320ks}
P=$PWD/respasol_amd/build/probe
for arm in ${ARMS:-"s4:RSP_ILU_FLOW_MODE=0" "t4:RSP_ILU_FLOW_MODE=2" "nosteal:RSP_PROBE_LIB=$P/nosteal/librsp.so" "bidx:RSP_PROBE_LIB=$P/bidx/librsp.so" "both:RSP_PROBE_LIB=$P/both/librsp.so"}; do
  name=${arm%%:*}; envs=${arm#*:}; [ "$envs" = "$arm" ] && envs=""
  env ${envs//,/ } timeout -k 10 300 python scripts/bench_ilu0.py --set $SET --fp64-only --reps 5 > $O/${name}.txt 2>&1 || exit 1
  echo "$name: $(grep TOTAL $O/${name}.txt | cut -c1-60)"
done
