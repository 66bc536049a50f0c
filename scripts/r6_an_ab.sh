# round 6: analysis A/B (current build vs a probe build), interleaved, one box
set -u
O=gpurun_out/${TAG:-r6anab}
mkdir -p $O
P=$PWD/respasol_amd/build/probe
for arm in cur prev cur2 prev2; do
  case $arm in prev*) env="RSP_PROBE_LIB=$P/prev/librsp.so";; *) env="";; esac
  env $env RSP_ILU_TIMING=1 timeout -k 10 300 python scripts/ilu_analysis_timing.py moderate 2 > $O/$arm.txt 2>&1 || exit 1
  echo "$arm: $(tail -1 $O/$arm.txt)"
done
