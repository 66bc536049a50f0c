#!/bin/bash
# Batched vs per-matrix launch A/B on one GPU, plus a 2-rank gloo rehearsal
# of the multi-GPU step (both ranks on the one GPU). Stops at the first failure.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=${1:-ab}
O=gpurun_out/$TAG
mkdir -p "$O"
export TMPDIR=/tmp
run() { local name=$1; shift; timeout -k 10 500 "$@" > "$O/$name.json" 2> "$O/$name.err"; local rc=$?;
        echo "$name rc=$rc"; [ $rc -eq 0 ] || { tail -20 "$O/$name.err"; exit $rc; }; }
[ -n "${TESTS:-}" ] && { timeout -k 10 600 python -m pytest $TESTS -q -x -rf > "$O/pytest.log" 2>&1;
    rc=$?; tail -5 "$O/pytest.log"; [ $rc -eq 0 ] || exit $rc; }
run big_batch python bench.py --steps 30 --warmup 3 --no-cpu
run big_eager python bench.py --steps 30 --warmup 3 --no-cpu --no-batch
run mod_batch python bench.py --steps 30 --warmup 3 --no-cpu --workload moderate
run n2_gloo python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
    --master-port 29511 bench.py --gpus 2 --steps 20 --warmup 3 --dist-backend gloo
for f in "$O"/*.json; do
    python - "$f" <<'PY'
import json, sys
for l in open(sys.argv[1]):
    if l.startswith("{"):
        d = json.loads(l)
        print(sys.argv[1].split("/")[-1], d["value"], d["ms_per_step"], d["roofline"]["frac"],
              d["roofline"]["avg_launch_us"], d["parity_check"], d["config"].get("launch"),
              d.get("per_matrix_calls"), d["fp32"])
PY
done
