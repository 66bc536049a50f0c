set -u
O=gpurun_out/${TAG:-r6t5}
mkdir -p $O
SET=${SET:-offshore,stomach,xenon2,para-10,2cubes_sphere,cfd2,FEM_3D_thermal2,Goodwin_095,tmt_unsym,ecology2,crashbasis,ASIC_320ks}
for r in 1; do
  for arm in "s4:RSP_ILU_FLOW_MODE=0" "t4:RSP_ILU_FLOW_MODE=2" "s8:RSP_ILU_FLOW_MODE=0 RSP_ILU_FLOW_WPC=8" "t8:RSP_ILU_FLOW_MODE=2 RSP_ILU_FLOW_WPC=8" "t16:RSP_ILU_FLOW_MODE=2 RSP_ILU_FLOW_WPC=16" "c4:RSP_ILU_FLOW_MODE=1"; do
    name=${arm%%:*}; envs=${arm#*:}
    env $envs timeout -k 10 300 python scripts/bench_ilu0.py --set $SET --fp64-only --reps 5 > $O/${name}_$r.txt 2>&1 || exit 1
    echo "$name $r: $(grep TOTAL $O/${name}_$r.txt | cut -c1-60)"
  done
done
