set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/${TAG:-r6pf}
mkdir -p $O
for m in 0 2; do
RSP_ILU_FLOW_MODE=$m timeout -k 10 300 rocprofv3 --kernel-trace -d $O/m$m -o run -- python3 scripts/ilu_kernel_probe.py ${NAMES:-offshore} > $O/m$m.log 2>&1 || { tail -30 $O/m$m.log; exit 1; }
grep rep $O/m$m.log
done
