#!/bin/bash
# A'-buffer sweeps restored (one wave), segment-parallel four-wave solve with the boundary system
# formed entry-parallel; 4 vs 2 segments; LOVE tile split; config-5 multiplier placement A/B.
set -e
OUT=gpurun_out/r3l
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p $OUT
LIB=$PWD/gp-mpc_amd/gpmpc/lib
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_launch.py tests/test_gpu_love.py -v --timeout 200 --timeout-method thread > $OUT/pytest_launch.log 2>&1 || { tail -80 $OUT/pytest_launch.log; exit 1; }
tail -2 $OUT/pytest_launch.log
GPMPC_LIB=$LIB/libgpmpc_mi355x_s2.so timeout -k 10 600 python3 -u -m pytest tests/test_gpu_launch.py -v --timeout 200 --timeout-method thread > $OUT/pytest_launch_s2.log 2>&1 || { tail -80 $OUT/pytest_launch_s2.log; exit 1; }
tail -2 $OUT/pytest_launch_s2.log
timeout -k 10 300 python3 -u bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline > $OUT/bench.json 2> $OUT/bench.err
for W in 1 4; do
GPMPC_WAVES=$W timeout -k 10 240 python3 -u bench.py --model cartpole --n-train 50 --horizon 20 --batch 256 --steps 20 --warmup 5 --no-cpu-baseline > $OUT/config2_w$W.json 2>> $OUT/bench.err
GPMPC_WAVES=$W timeout -k 10 240 python3 -u bench.py --batch 256 --steps 20 --warmup 5 --no-cpu-baseline > $OUT/c3b256_w$W.json 2>> $OUT/bench.err
done
GPMPC_LIB=$LIB/libgpmpc_mi355x_s2.so GPMPC_WAVES=4 timeout -k 10 240 python3 -u bench.py --model cartpole --n-train 50 --horizon 20 --batch 256 --steps 20 --warmup 5 --no-cpu-baseline > $OUT/config2_s2.json 2>> $OUT/bench.err
GPMPC_LIB=$LIB/libgpmpc_mi355x_s2.so GPMPC_WAVES=4 timeout -k 10 240 python3 -u bench.py --batch 256 --steps 20 --warmup 5 --no-cpu-baseline > $OUT/c3b256_s2.json 2>> $OUT/bench.err
timeout -k 10 120 python3 tools/phase_timing.py --batch 256 --warmup 5 --waves 4 > $OUT/ph_c3b256_w4.txt 2>&1
GPMPC_LIB=$LIB/libgpmpc_mi355x_s2_timing.so timeout -k 10 120 python3 tools/phase_timing.py --batch 256 --warmup 5 --waves 4 > $OUT/ph_c3b256_s2.txt 2>&1
C5="--model quad3d --n-train 4000 --fitc 2000 --horizon 40 --batch 512 --var-inputs dynamics --steps 10 --warmup 3 --no-cpu-baseline"
timeout -k 10 400 python3 -u bench.py $C5 > $OUT/c5_cur.json 2>> $OUT/bench.err
GPMPC_LIB=$LIB/libgpmpc_mi355x_q3g.so timeout -k 10 400 python3 -u bench.py $C5 > $OUT/c5_q3g.json 2>> $OUT/bench.err
GPMPC_LIB=$LIB/libgpmpc_mi355x_r2k.so timeout -k 10 400 python3 -u bench.py $C5 > $OUT/c5_r2k.json 2>> $OUT/bench.err
python3 - <<'PY'
import json
for f in ["bench", "config2_w1", "config2_w4", "config2_s2", "c3b256_w1", "c3b256_w4", "c3b256_s2", "c5_cur", "c5_q3g", "c5_r2k"]:
    d = json.loads([x for x in open(f"gpurun_out/r3l/{f}.json") if x.startswith("{")][-1])
    print(f, round(d["value"]), d["kernel_ms_per_step"], d["sqp_iter_mean"], d["qp_iter_mean_per_step"], d["status_counts"])
PY
grep -v amdgpu.ids $OUT/ph_*.txt
