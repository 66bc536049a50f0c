# flow launches: static walk vs start tickets (lookahead 4 / probe build) on the FEM solves
set -u
O=gpurun_out/${TAG:-r6t}
mkdir -p $O
SET=${SET:-offshore,stomach,xenon2,para-10,2cubes_sphere,cfd2,FEM_3D_thermal2,Goodwin_095,tmt_unsym,ecology2,crashbasis,ASIC_320ks}
for r in 1 2; do
  RSP_ILU_FLOW_MODE=0 timeout -k 10 300 python scripts/bench_ilu0.py --set $SET --fp64-only --reps 5 > $O/static_$r.txt 2>&1 || exit 1
  RSP_ILU_FLOW_MODE=2 timeout -k 10 300 python scripts/bench_ilu0.py --set $SET --fp64-only --reps 5 > $O/t4_$r.txt 2>&1 || exit 1
  for k in ${KS:-16}; do RSP_PROBE_LIB=$PWD/respasol_amd/build/probe/ahead$k/librsp.so RSP_ILU_FLOW_MODE=2 timeout -k 10 300 python scripts/bench_ilu0.py --set $SET --fp64-only --reps 5 > $O/t${k}_$r.txt 2>&1 || exit 1; done
  for a in static t4 $(for k in ${KS:-16}; do echo t$k; done); do echo "$a $r: $(grep TOTAL $O/${a}_$r.txt | cut -c1-60)"; done
done
