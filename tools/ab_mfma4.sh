#!/bin/bash
# Variance kernels' 16x16x4 f64 tiles as four v_mfma_f64_4x4x4_4b_f64 (round 3): the GPU suite on
# the new library, then configs 3/4/5/2 against the previous commit's library (ord16).
set -e
OUT=gpurun_out/mfma4
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p $OUT
LIB=$PWD/gp-mpc_amd/gpmpc/lib
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_love.py tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread > $OUT/pytest_var.log 2>&1 || { tail -40 $OUT/pytest_var.log; exit 1; }
tail -1 $OUT/pytest_var.log
A="--steps 20 --warmup 5 --no-cpu-baseline"
C2="--model cartpole --n-train 50 --horizon 20 --batch 256"
C4="--n-train 1000"
C5="--model quad3d --n-train 4000 --fitc 2000 --horizon 40 --batch 512 --var-inputs dynamics"
for V in new ord16; do
L=$LIB/libgpmpc_mi355x.so; [ $V != new ] && L=$LIB/libgpmpc_mi355x_$V.so
for c in 3 4 5 2; do
  eval ARGS=\$C$c
  [ $c = 3 ] && ARGS=""
  GPMPC_LIB=$L timeout -k 10 300 python3 -u bench.py $ARGS $A > $OUT/c${c}_$V.json 2>> $OUT/bench.err
done
done
python3 - <<'PY'
import json
for c in [3, 4, 5, 2]:
    for V in ["new", "ord16"]:
        d = json.loads([x for x in open(f"gpurun_out/mfma4/c{c}_{V}.json") if x.startswith("{")][-1])
        rv = d.get("roofline_variance", {})
        print(c, V, round(d["value"]), {k: round(v, 4) for k, v in d["kernel_ms_per_step"].items()}, round(d["sqp_iter_mean"], 4),
              d["status_counts"]["0"], round(rv.get("achieved", 0), 1))
PY
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || { tail -40 $OUT/pytest_gpu.log; exit 1; }
tail -1 $OUT/pytest_gpu.log
