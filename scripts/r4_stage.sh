#!/bin/bash
# Round 4: staged SpMV tiles — parity, per-matrix A/B (variant 1024 = no
# staging), batched bench step A/B.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/${1:-r4stage}
mkdir -p "$O"
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_spmv.py tests/test_gpu_spmv_batch.py tests/test_gpu_fullsize.py -q -x -rf \
    -k "${PYK:-not ilu}" --timeout 300 --timeout-method thread > "$O/pytest.log" 2>&1
rc=$?; tail -3 "$O/pytest.log"; [ $rc -eq 0 ] || exit $rc
for dt in f64 f32; do
    timeout -k 10 300 python scripts/spmv_ab.py --variants 0,1024 --dtype $dt --rounds 3 > "$O/ab_$dt.txt" 2>&1 || { tail -5 "$O/ab_$dt.txt"; exit 1; }
    tail -2 "$O/ab_$dt.txt"
done
for r in 1 2; do
    for v in 0 1024; do
        RSP_SPMV_VARIANT=$v timeout -k 10 300 python bench.py --no-cpu --no-config5 > "$O/bench_v${v}_$r.json" 2> "$O/bench_v${v}_$r.err" || { tail -5 "$O/bench_v${v}_$r.err"; exit 1; }
        python3 -c "import json,sys; d=json.loads(open('$O/bench_v${v}_$r.json').read().strip().splitlines()[-1]); print('v$v', d['value'], d['ms_per_step'], d['roofline']['frac'], 'fp32', d['fp32']['ms_per_pass_rank0'], d['fp32']['roofline']['frac'])"
    done
done
