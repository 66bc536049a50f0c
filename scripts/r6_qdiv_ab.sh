# round 6: FTZ division variants (probe builds) on the factor, then the FTZ parity tests
set -u
O=gpurun_out/${TAG:-r6q}
mkdir -p $O
P=$PWD/respasol_amd/build/probe
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "ftz or Ftz or FTZ or division" > $O/pytest_ftz.txt 2>&1 || { tail -30 $O/pytest_ftz.txt; exit 1; }
tail -1 $O/pytest_ftz.txt
SET=dc1,matrix-new_3,xenon2,ASIC_320ks,crashbasis
for arm in "cur:" "plain:RSP_PROBE_LIB=$P/plain/librsp.so" "f64:RSP_PROBE_LIB=$P/f64/librsp.so" "cur2:"; do
  name=${arm%%:*}; envs=${arm#*:}
  env $envs timeout -k 10 300 python scripts/bench_ilu0.py --set $SET --reps 5 > $O/${name}.txt 2>&1 || exit 1
  echo "$name: $(grep TOTAL $O/${name}.txt)"
done
