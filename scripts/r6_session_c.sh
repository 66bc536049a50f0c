# round 6: start tickets with steals — flow tests, then static vs ticket A/B
set -u
O=gpurun_out/${TAG:-r6c}
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_ilu0.py -x -v --timeout 120 --timeout-method thread -k "flow" > $O/pytest_flow.txt 2>&1 || { tail -30 $O/pytest_flow.txt; exit 1; }
tail -3 $O/pytest_flow.txt
SET=${SET:-offshore,stomach,xenon2,para-10,2cubes_sphere,cfd2,FEM_3D_thermal2,Goodwin_095,tmt_unsym,ecology2,crashbasis,ASIC_320ks}
for arm in "s4:RSP_ILU_FLOW_MODE=0" "t4:RSP_ILU_FLOW_MODE=2" "s8:RSP_ILU_FLOW_MODE=0 RSP_ILU_FLOW_WPC=8" "t8:RSP_ILU_FLOW_MODE=2 RSP_ILU_FLOW_WPC=8"; do
  name=${arm%%:*}; envs=${arm#*:}
  env $envs timeout -k 10 300 python scripts/bench_ilu0.py --set $SET --fp64-only --reps 5 > $O/${name}.txt 2>&1 || exit 1
  echo "$name: $(grep TOTAL $O/${name}.txt | cut -c1-60)"
done
