#!/bin/bash
# Quick iteration pass on one MI355X (run through gpurun from the repo root):
#   bash tools/gpu_iter.sh OUTDIR
# 1. tools/ric_micro (sweep micro-benchmarks + MFMA4-vs-VALU check), if built
# 2. the GPU parity tests  3. bench.py at the driver's command (no CPU baseline)
set -e
OUT=${1:?outdir}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p "$OUT"
if [ -x tools/ric_micro ]; then timeout -k 10 120 ./tools/ric_micro > "$OUT/ric_micro.txt" 2>&1; cat "$OUT/ric_micro.txt"; fi
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > "$OUT/pytest_gpu.log" 2>&1 || { tail -30 "$OUT/pytest_gpu.log"; exit 1; }
tail -3 "$OUT/pytest_gpu.log"
timeout -k 10 300 python3 -u bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline > "$OUT/bench.json" 2> "$OUT/bench.err"
python3 -c "import json; d=json.load(open('$OUT/bench.json')); print('value', round(d['value']), 'ms/step', round(d['ms_per_step'],4), 'sqp', round(d['kernel_ms_per_step']['sqp'],4), 'var', round(d['kernel_ms_per_step']['variance'],4), 'sqp it', d['sqp_iter_mean'], d['sqp_iter_max'], 'qp', d['qp_iter_mean_per_step'], d['qp_iter_max_per_step'], 'status', d['status_counts'])"
