# round 6: FTZ division without mode switches — FTZ parity tests + config-3 bench
set -u
O=gpurun_out/${TAG:-r6ftz}
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "ftz or Ftz or FTZ or fullsize or division" > $O/pytest_ftz.txt 2>&1 || { tail -30 $O/pytest_ftz.txt; exit 1; }
tail -2 $O/pytest_ftz.txt
timeout -k 10 600 python scripts/bench_ilu0.py --reps 3 --json $O/ilu_config3.json > $O/ilu_config3.txt 2> $O/ilu_config3.err || exit 1
tail -1 $O/ilu_config3.txt
RSP_ILU_TIMING=1 timeout -k 10 300 python scripts/ilu_analysis_timing.py moderate 2 > $O/an_timing.txt 2>&1 || exit 1
tail -1 $O/an_timing.txt
