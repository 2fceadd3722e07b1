#!/bin/bash
# Round-3 check of the condensed Riccati path and the multi-wave launch: the launch-shape parity tests
# (every combination, no -x), the whole GPU suite, then the driver's bench command with and without
# condensing (GPMPC_CONDENSE=0), config 2 with each launch shape, and config 5.
set -e
OUT=gpurun_out/r3c
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p $OUT
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_launch.py -v --timeout 200 --timeout-method thread > $OUT/pytest_launch.log 2>&1 || { tail -60 $OUT/pytest_launch.log; exit 1; }
tail -3 $OUT/pytest_launch.log
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || { tail -40 $OUT/pytest_gpu.log; exit 1; }
tail -3 $OUT/pytest_gpu.log
timeout -k 10 300 python3 -u bench.py --gpus 1 --steps 20 --warmup 5 > $OUT/bench.json 2> $OUT/bench.err
GPMPC_CONDENSE=0 timeout -k 10 300 python3 -u bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline > $OUT/bench_nocond.json 2> $OUT/bench_nocond.err
for W in 1 4; do for C in 0 1; do
GPMPC_WAVES=$W GPMPC_CONDENSE=$C timeout -k 10 240 python3 -u bench.py --model cartpole --n-train 50 --horizon 20 --batch 256 --steps 20 --warmup 5 --no-cpu-baseline > $OUT/config2_w${W}c${C}.json 2>> $OUT/bench.err
done; done
timeout -k 10 600 python3 -u bench.py --model quad3d --n-train 4000 --fitc 2000 --horizon 40 --batch 512 --var-inputs dynamics --steps 20 --warmup 5 --no-cpu-baseline > $OUT/config5.json 2>> $OUT/bench.err
python3 - <<'PY'
import json
for f in ["bench", "bench_nocond", "config2_w1c0", "config2_w1c1", "config2_w4c0", "config2_w4c1", "config5"]:
    d = json.loads([x for x in open(f"gpurun_out/r3c/{f}.json") if x.startswith("{")][-1])
    print(f, round(d["value"]), d["kernel_ms_per_step"], d["sqp_iter_mean"], d["qp_iter_mean_per_step"], d["status_counts"])
PY
