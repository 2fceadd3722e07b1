#!/bin/bash
# Cost-ordered dispatch A/B (round 3): config 5 (512 instances, one per CU: two rounds) with the
# ordering on / off (GPMPC_ORDER=0) and the previous commit's library; config 3 (one round, no
# ordering) against the previous library; then the GPU test suite.
set -e
OUT=gpurun_out/order
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p $OUT
LIB=$PWD/gp-mpc_amd/gpmpc/lib
A="--steps 20 --warmup 5 --no-cpu-baseline"
C5="--model quad3d --n-train 4000 --fitc 2000 --horizon 40 --batch 512 --var-inputs dynamics"
timeout -k 10 300 python3 -u bench.py $C5 $A > $OUT/c5_order.json 2> $OUT/c5_order.err
GPMPC_ORDER=0 timeout -k 10 300 python3 -u bench.py $C5 $A > $OUT/c5_noorder.json 2> $OUT/c5_noorder.err
GPMPC_LIB=$LIB/libgpmpc_mi355x_head.so timeout -k 10 300 python3 -u bench.py $C5 $A > $OUT/c5_head.json 2> $OUT/c5_head.err
for r in 1 2; do
timeout -k 10 200 python3 -u bench.py $A > $OUT/c3_new_$r.json 2> $OUT/c3_new.err
GPMPC_LIB=$LIB/libgpmpc_mi355x_head.so timeout -k 10 200 python3 -u bench.py $A > $OUT/c3_head_$r.json 2> $OUT/c3_head.err
done
python3 - <<'PY'
import json, glob
for f in sorted(glob.glob("gpurun_out/order/*.json")):
    d = json.loads([x for x in open(f) if x.startswith("{")][-1])
    print(f.split("/")[-1], round(d["value"]), d["kernel_ms_per_step"], d["sqp_iter_mean"], d["status_counts"],
          d["sqp_kernel_ms_per_step_distribution"]["p50"])
PY
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || { tail -40 $OUT/pytest_gpu.log; exit 1; }
tail -3 $OUT/pytest_gpu.log
