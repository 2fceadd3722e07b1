#!/bin/bash
# Strong scaling of the metric's global batch (config 3, 1024 instances) from one GPU (run through
# gpurun from the repo root): bash tools/shard_sweep.sh OUTDIR [extra bench args...]
# For N = 1, 2, 4, 8 every rank's contiguous slice of the global batch runs alone on the GPU
# (bench.py --shard R/N: the same instance ids, initial states and reference phases as rank R of
# `bench.py --gpus N`, which has no collective in the step); the job's step time is its slowest
# shard's, so the projected job value is 1024 x steps / max over shards of the shard's time.
set -e
OUT=${1:?outdir}
shift
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p "$OUT"
for N in 1 2 4 8; do
  for R in $(seq 0 $((N - 1))); do
    timeout -k 10 180 python3 -u bench.py --shard $R/$N --steps 20 --warmup 5 --no-cpu-baseline "$@" \
        > "$OUT/n${N}_r${R}.json" 2> "$OUT/n${N}_r${R}.err"
  done
done
python3 - "$OUT" <<'PY'
import json, sys
out = sys.argv[1]
base = None
print("GPUs  instances/GPU  slowest shard ms/step (SQP / var)  fastest shard  projected job steps/s  speed-up")
for N in (1, 2, 4, 8):
    ds = [json.loads([x for x in open(f"{out}/n{N}_r{R}.json") if x.startswith("{")][-1]) for R in range(N)]
    slow = max(ds, key=lambda d: d["ms_per_step"])
    fast = min(d["ms_per_step"] for d in ds)
    val = 1024 / (slow["ms_per_step"] * 1e-3)
    base = base or val
    print(f"{N:4d}  {slow['config']['batch_per_gpu']:13d}  {slow['ms_per_step']:.4f} ({slow['kernel_ms_per_step']['sqp']:.4f} / "
          f"{slow['kernel_ms_per_step']['variance']:.4f})  rank {slow['emulated_shard']['rank']}   {fast:.4f}   "
          f"{val:12.0f}   {val / base:.2f}")
PY
