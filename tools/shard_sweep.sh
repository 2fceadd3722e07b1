#!/bin/bash
# Per-GPU time of each strong-scaled shard of the metric's global batch (run through gpurun from the
# repo root): bash tools/shard_sweep.sh OUTDIR [extra bench args...]
# Config 3 (quad2d N=200 H=30) on one GPU with B = 1024/N instances for N = 8, 4, 2, 1: the time one
# rank of `bench.py --gpus N --global-batch 1024` spends per step (no collective in the step).
set -e
OUT=${1:?outdir}
shift
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p "$OUT"
for B in 128 256 512 1024; do
  timeout -k 10 180 python3 -u bench.py --gpus 1 --steps 20 --warmup 5 --batch $B --no-cpu-baseline "$@" \
      > "$OUT/b$B.json" 2> "$OUT/b$B.err"
done
python3 - "$OUT" <<'PY'
import json, sys
out = sys.argv[1]
for B in (128, 256, 512, 1024):
    d = json.loads([x for x in open(f"{out}/b{B}.json") if x.startswith("{")][-1])
    print(f"B={B:5d} ms/step {d['ms_per_step']:.4f}  sqp {d['kernel_ms_per_step']['sqp']:.4f}  var {d['kernel_ms_per_step']['variance']:.4f}  value {d['value']:.0f}  sqp_iter {d['sqp_iter_mean']:.3f}")
PY
