#!/bin/bash
# Round profiling session on the GPU box; every summary bench.py's roofline
# cites comes from here (copy with scripts/collect_profiles.py):
#   1. rocprofv3 --kernel-trace --stats on the DRIVER'S OWN bench command
#      (python3 bench.py --gpus 1 --steps 20 --warmup 5: clock ramp, warm-up,
#      timed steps, config-5 Serena step, CPU baseline, all as the driver runs
#      it) -> stats/ + bench_prof.json; scripts/check_roofline.py then checks
#      that the rocprof average of spmv_tiles_batch<double> agrees with the
#      line's avg_launch_us
#   2. rocprofv3 --pmc FETCH_SIZE on scripts/pmc_run.py (own run; fp64 then fp32)
#   3. rocprofv3 --pmc WRITE_SIZE on scripts/pmc_run.py (own run)
#   4. scripts/pmc_summary.py -> <tag>_pmc.json stamped with the kernel
#      source hash (bench.py refuses a summary of another build) and the
#      commit (RSP_COMMIT, passed in the gpurun command: the box has no .git)
# Each GPU step has its own time limit; stop at the first fault/timeout.
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
TAG=${1:-r03}
OUT="$ROOT/gpurun_out/$TAG"
mkdir -p "$OUT"
export TMPDIR=/tmp
cd /tmp
fatal() { if [ "$1" -ne 0 ]; then echo "STOP: $2 exited $1"; exit "$1"; fi; }
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/stats" -o run -- \
    python3 "$ROOT/bench.py" --gpus 1 --steps 20 --warmup 5 > "$OUT/bench_prof.json" 2> "$OUT/stats.err"
rc=$?; echo "stats rc=$rc"; fatal $rc stats
timeout -k 10 600 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$OUT/fetch" -o run -- \
    python3 "$ROOT/scripts/pmc_run.py" --meta "$OUT/meta.json" > "$OUT/fetch.log" 2>&1
rc=$?; echo "fetch rc=$rc"; fatal $rc fetch
timeout -k 10 600 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$OUT/write" -o run -- \
    python3 "$ROOT/scripts/pmc_run.py" > "$OUT/write.log" 2>&1
rc=$?; echo "write rc=$rc"; fatal $rc write
cd "$ROOT"
python3 scripts/pmc_summary.py --fetch "$OUT/fetch" --write "$OUT/write" --meta "$OUT/meta.json" \
    --out "$OUT/${TAG}_pmc.json"
python3 scripts/pmc_summary.py --fetch "$OUT/fetch" --write "$OUT/write" --meta "$OUT/meta.json" \
    --dtype f32 --out "$OUT/${TAG}_pmc_f32.json"
python3 scripts/check_roofline.py --stats "$OUT/stats" --bench "$OUT/bench_prof.json" | tee "$OUT/roofline_check.txt"
python3 scripts/check_roofline.py --fp32 --stats "$OUT/stats" --bench "$OUT/bench_prof.json" | tee -a "$OUT/roofline_check.txt"
