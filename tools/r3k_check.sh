#!/bin/bash
# Double-buffered sweep operands (one wave) and the segment boundaries on wave 1 (four waves).
set -e
OUT=gpurun_out/r3k
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p $OUT
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_launch.py -v --timeout 200 --timeout-method thread > $OUT/pytest_launch.log 2>&1 || { tail -80 $OUT/pytest_launch.log; exit 1; }
tail -2 $OUT/pytest_launch.log
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_love.py -v --timeout 200 --timeout-method thread > $OUT/pytest_love.log 2>&1 || { tail -80 $OUT/pytest_love.log; exit 1; }
tail -2 $OUT/pytest_love.log
timeout -k 10 300 python3 -u bench.py --n-train 1000 --steps 20 --warmup 5 --no-cpu-baseline > $OUT/config4.json 2>> $OUT/bench.err
timeout -k 10 300 python3 -u tools/love_split.py > $OUT/love_split.txt 2>&1
timeout -k 10 300 python3 -u bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline > $OUT/bench.json 2> $OUT/bench.err
for W in 1 4; do
GPMPC_WAVES=$W timeout -k 10 240 python3 -u bench.py --model cartpole --n-train 50 --horizon 20 --batch 256 --steps 20 --warmup 5 --no-cpu-baseline > $OUT/config2_w$W.json 2>> $OUT/bench.err
GPMPC_WAVES=$W timeout -k 10 240 python3 -u bench.py --batch 256 --steps 20 --warmup 5 --no-cpu-baseline > $OUT/c3b256_w$W.json 2>> $OUT/bench.err
done
timeout -k 10 120 python3 tools/phase_timing.py --warmup 5 > $OUT/ph_c3.txt 2>&1
timeout -k 10 120 python3 tools/phase_timing.py --model cartpole --n-train 50 --horizon 20 --batch 256 --warmup 5 --waves 4 > $OUT/ph_c2_w4.txt 2>&1
timeout -k 10 120 python3 tools/phase_timing.py --batch 256 --warmup 5 --waves 4 > $OUT/ph_c3b256_w4.txt 2>&1
timeout -k 10 120 python3 tools/phase_timing.py --batch 256 --warmup 5 --waves 1 > $OUT/ph_c3b256_w1.txt 2>&1
python3 - <<'PY'
import json
for f in ["config4", "bench", "config2_w1", "config2_w4", "c3b256_w1", "c3b256_w4"]:
    d = json.loads([x for x in open(f"gpurun_out/r3k/{f}.json") if x.startswith("{")][-1])
    print(f, round(d["value"]), d["kernel_ms_per_step"], d["sqp_iter_mean"], d["qp_iter_mean_per_step"], d["status_counts"])
PY
grep -v amdgpu.ids $OUT/ph_*.txt $OUT/love_split.txt
