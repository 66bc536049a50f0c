#!/bin/bash
# Env-knob A/B on the bench step (batched, big set; then the
# moderate set): "name:ENV=... " specs, interleaved rounds.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/${1:-benchab}; shift
mkdir -p "$O"
export TMPDIR=/tmp
for wl in ${WORKLOADS:-big}; do
for r in $(seq 1 "${ROUNDS:-2}"); do
    for spec in "$@"; do
        name=${spec%%:*}; envs=${spec#*:}
        env $envs timeout -k 10 300 python bench.py --no-cpu --no-config5 --workload $wl > "$O/${wl}_${name}_$r.json" 2> "$O/${wl}_${name}_$r.err" \
            || { tail -5 "$O/${wl}_${name}_$r.err"; exit 1; }
        python3 -c "import json; d=json.loads(open('$O/${wl}_${name}_$r.json').read().strip().splitlines()[-1]); print('$wl $name', d['value'], d['ms_per_step'], d['roofline']['frac'], 'fp32', d['fp32']['ms_per_pass_rank0'], d['fp32']['roofline']['frac'], 'calls', d['per_matrix_calls']['ms_per_step_rank0'])"
    done
done
done
