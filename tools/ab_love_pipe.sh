#!/bin/bash
# LOVE kernel with compile-time tile counts (new, the K loop branch-free) and with the next K-step's
# exp interleaved between MFMAs (sched, -DGPMPC_LOVE_SCHED) against the previous library (base):
# LOVE parity on each, then configs 4 and 5 (round 3).
set -e
OUT=gpurun_out/lovepipe
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p $OUT
LIB=$PWD/gp-mpc_amd/gpmpc/lib
for V in new sched; do
L=$LIB/libgpmpc_mi355x.so; [ $V != new ] && L=$LIB/libgpmpc_mi355x_$V.so
GPMPC_LIB=$L timeout -k 10 300 python3 -u -m pytest tests/test_gpu_love.py -x -q --timeout 200 --timeout-method thread > $OUT/pytest_$V.log 2>&1 || { tail -40 $OUT/pytest_$V.log; exit 1; }
tail -1 $OUT/pytest_$V.log
done
A="--steps 20 --warmup 5 --no-cpu-baseline"
C4="--n-train 1000"
C5="--model quad3d --n-train 4000 --fitc 2000 --horizon 40 --batch 512 --var-inputs dynamics"
for r in 1 2; do
for V in new sched base; do
L=$LIB/libgpmpc_mi355x.so; [ $V != new ] && L=$LIB/libgpmpc_mi355x_$V.so
GPMPC_LIB=$L timeout -k 10 300 python3 -u bench.py $C4 $A > $OUT/c4_${V}_$r.json 2>> $OUT/bench.err
[ $r = 1 ] && GPMPC_LIB=$L timeout -k 10 300 python3 -u bench.py $C5 $A > $OUT/c5_${V}.json 2>> $OUT/bench.err
done
done
python3 - <<'PY'
import json, glob
for f in sorted(glob.glob("gpurun_out/lovepipe/c*.json")):
    d = json.loads([x for x in open(f) if x.startswith("{")][-1])
    rv = d.get("roofline_variance", {})
    print(f.split("/")[-1], round(d["value"]), {k: round(v, 4) for k, v in d["kernel_ms_per_step"].items()}, round(rv.get("achieved", 0), 1))
PY
