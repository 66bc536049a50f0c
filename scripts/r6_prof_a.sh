set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/${TAG:-r6p}
mkdir -p $O
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/blk -o run -- python3 scripts/ilu_kernel_probe.py dc1 G2_circuit > $O/blk.log 2>&1 || { tail -30 $O/blk.log; exit 1; }
grep rep $O/blk.log
RSP_ILU_FLOW_MODE=0 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/static -o run -- python3 scripts/ilu_kernel_probe.py offshore stomach > $O/static.log 2>&1 || { tail -30 $O/static.log; exit 1; }
grep rep $O/static.log
RSP_ILU_FLOW_MODE=2 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/ticket -o run -- python3 scripts/ilu_kernel_probe.py offshore stomach > $O/ticket.log 2>&1 || { tail -30 $O/ticket.log; exit 1; }
grep rep $O/ticket.log
find $O -name "*stats*"
