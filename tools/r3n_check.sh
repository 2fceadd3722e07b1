#!/bin/bash
# Segment-parallel four-wave solve with the register-resident boundary chain (variant libraries
# built from the round-3 segment patch) against the shipped four-wave kernel (GP helpers only).
set -e
OUT=gpurun_out/r3n
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p $OUT
LIB=$PWD/gp-mpc_amd/gpmpc/lib
for V in s4 s2; do
GPMPC_LIB=$LIB/libgpmpc_mi355x_$V.so timeout -k 10 600 python3 -u -m pytest tests/test_gpu_launch.py -v --timeout 200 --timeout-method thread > $OUT/pytest_launch_$V.log 2>&1 || { tail -60 $OUT/pytest_launch_$V.log; exit 1; }
tail -1 $OUT/pytest_launch_$V.log
done
A="--steps 20 --warmup 5 --no-cpu-baseline"
C2="--model cartpole --n-train 50 --horizon 20 --batch 256"
for V in prod s4 s2; do
L=$LIB/libgpmpc_mi355x.so; [ $V != prod ] && L=$LIB/libgpmpc_mi355x_$V.so
GPMPC_LIB=$L timeout -k 10 240 python3 -u bench.py $C2 $A > $OUT/config2_$V.json 2>> $OUT/bench.err
GPMPC_LIB=$L timeout -k 10 240 python3 -u bench.py --batch 256 $A > $OUT/c3b256_$V.json 2>> $OUT/bench.err
GPMPC_LIB=$L timeout -k 10 240 python3 -u bench.py --batch 128 $A > $OUT/c3b128_$V.json 2>> $OUT/bench.err
done
GPMPC_LIB=$LIB/libgpmpc_mi355x_s4_timing.so timeout -k 10 120 python3 tools/phase_timing.py --batch 256 --warmup 5 --waves 4 > $OUT/ph_c3b256_s4.txt 2>&1
timeout -k 10 120 python3 tools/phase_timing.py --batch 256 --warmup 5 --waves 4 > $OUT/ph_c3b256_prod.txt 2>&1
python3 - <<'PY'
import json
for V in ["prod", "s4", "s2"]:
    for f in ["config2", "c3b256", "c3b128"]:
        d = json.loads([x for x in open(f"gpurun_out/r3n/{f}_{V}.json") if x.startswith("{")][-1])
        print(f, V, round(d["value"]), d["kernel_ms_per_step"], d["sqp_iter_mean"], d["status_counts"])
PY
grep -v amdgpu.ids $OUT/ph_*.txt
