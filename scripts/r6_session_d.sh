# round 6: old (HEAD~ probe build) vs new flow walk on one box
set -u
O=gpurun_out/${TAG:-r6d}
mkdir -p $O
SET=${SET:-offshore,stomach,xenon2,para-10,2cubes_sphere,cfd2,FEM_3D_thermal2,Goodwin_095,tmt_unsym,ecology2,crashbasis,ASIC_320ks}
OLD=$PWD/respasol_amd/build/probe/old/librsp.so
for arm in "olds4:RSP_PROBE_LIB=$OLD RSP_ILU_FLOW_MODE=0" "news4:RSP_ILU_FLOW_MODE=0" "newt4:RSP_ILU_FLOW_MODE=2" "oldt4:RSP_PROBE_LIB=$OLD RSP_ILU_FLOW_MODE=2" "news4b:RSP_ILU_FLOW_MODE=0" "newt4b:RSP_ILU_FLOW_MODE=2" ${EXTRA_ARMS:-}; do
  name=${arm%%:*}; envs=${arm#*:}
  env $envs timeout -k 10 300 python scripts/bench_ilu0.py --set $SET --fp64-only --reps 5 > $O/${name}.txt 2>&1 || exit 1
  echo "$name: $(grep TOTAL $O/${name}.txt | cut -c1-60)"
done
