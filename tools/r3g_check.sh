#!/bin/bash
# Condensed path (revised) check: launch-shape parity, the GPU suite, benches and phase timings.
set -e
OUT=gpurun_out/r3g
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p $OUT
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_launch.py -v --timeout 200 --timeout-method thread > $OUT/pytest_launch.log 2>&1 || { tail -60 $OUT/pytest_launch.log; exit 1; }
tail -2 $OUT/pytest_launch.log
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || { tail -40 $OUT/pytest_gpu.log; exit 1; }
tail -2 $OUT/pytest_gpu.log
for C in 1 0; do
GPMPC_CONDENSE=$C timeout -k 10 300 python3 -u bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline > $OUT/bench_c$C.json 2> $OUT/bench.err
done
for W in 1 4; do for C in 0 1; do
GPMPC_WAVES=$W GPMPC_CONDENSE=$C timeout -k 10 240 python3 -u bench.py --model cartpole --n-train 50 --horizon 20 --batch 256 --steps 20 --warmup 5 --no-cpu-baseline > $OUT/config2_w${W}c${C}.json 2>> $OUT/bench.err
done; done
timeout -k 10 120 python3 tools/phase_timing.py --warmup 5 --waves 1 --condense > $OUT/ph_c3_w1c1.txt 2>&1
timeout -k 10 120 python3 tools/phase_timing.py --model cartpole --n-train 50 --horizon 20 --batch 256 --warmup 5 --waves 1 --condense > $OUT/ph_c2_w1c1.txt 2>&1
python3 - <<'PY'
import json
for f in ["bench_c1", "bench_c0", "config2_w1c0", "config2_w1c1", "config2_w4c0", "config2_w4c1"]:
    d = json.loads([x for x in open(f"gpurun_out/r3g/{f}.json") if x.startswith("{")][-1])
    print(f, round(d["value"]), d["kernel_ms_per_step"], d["sqp_iter_mean"], d["qp_iter_mean_per_step"], d["status_counts"])
PY
cat $OUT/ph_*.txt | grep -v amdgpu.ids
