#!/bin/bash
# Multipliers in LDS for the stage-by-stage MFMA path (A' formed on the fly in the sweeps):
# launch-shape parity, the GPU suite, config 3 / config 2 benches, phase timing, HBM traffic.
set -e
OUT=gpurun_out/r3i
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p $OUT
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_launch.py -v --timeout 200 --timeout-method thread > $OUT/pytest_launch.log 2>&1 || { tail -60 $OUT/pytest_launch.log; exit 1; }
tail -2 $OUT/pytest_launch.log
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || { tail -40 $OUT/pytest_gpu.log; exit 1; }
tail -2 $OUT/pytest_gpu.log
timeout -k 10 300 python3 -u bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline > $OUT/bench.json 2> $OUT/bench.err
timeout -k 10 240 python3 -u bench.py --model cartpole --n-train 50 --horizon 20 --batch 256 --steps 20 --warmup 5 --no-cpu-baseline > $OUT/config2.json 2>> $OUT/bench.err
timeout -k 10 120 python3 tools/phase_timing.py --warmup 5 > $OUT/ph_c3.txt 2>&1
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d "$OUT/fetch" -o run -- \
    python3 bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline > "$OUT/fetch.log" 2>&1
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d "$OUT/write" -o run -- \
    python3 bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline > "$OUT/write.log" 2>&1
python3 tools/pmc_summary.py --trace "$OUT/fetch" --fetch "$OUT/fetch" --write "$OUT/write" --last 20 \
    --config '{"workload": "r3i"}' -o "$OUT/pmc_summary.json"
python3 - <<'PY'
import json
for f in ["bench", "config2"]:
    d = json.loads([x for x in open(f"gpurun_out/r3i/{f}.json") if x.startswith("{")][-1])
    print(f, round(d["value"]), d["kernel_ms_per_step"], d["sqp_iter_mean"], d["qp_iter_mean_per_step"], d["status_counts"])
s = json.load(open("gpurun_out/r3i/pmc_summary.json"))
for k, v in s["kernels"].items():
    if "sqp" in k:
        print(k[:60], v["duration"]["mean_us"], v.get("FETCH_SIZE_kB"), v.get("WRITE_SIZE_kB"), v.get("hbm_bytes_est"))
PY
grep -v amdgpu.ids $OUT/ph_c3.txt
