#!/bin/bash
# Branch-free LOVE kernel with its 16x16x4 tiles as four v_mfma_f64_4x4x4_4b (by4, A quads by
# ds_swizzle) against the shipped 16x16x4 form (new): LOVE parity, configs 4 and 5 (round 3).
set -e
OUT=gpurun_out/loveby4
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p $OUT
LIB=$PWD/gp-mpc_amd/gpmpc/lib
GPMPC_LIB=$LIB/libgpmpc_mi355x_by4.so timeout -k 10 300 python3 -u -m pytest tests/test_gpu_love.py -x -q --timeout 200 --timeout-method thread > $OUT/pytest_by4.log 2>&1 || { tail -40 $OUT/pytest_by4.log; exit 1; }
tail -1 $OUT/pytest_by4.log
A="--steps 20 --warmup 5 --no-cpu-baseline"
C4="--n-train 1000"
C5="--model quad3d --n-train 4000 --fitc 2000 --horizon 40 --batch 512 --var-inputs dynamics"
for r in 1 2; do
for V in new by4; do
L=$LIB/libgpmpc_mi355x.so; [ $V != new ] && L=$LIB/libgpmpc_mi355x_$V.so
GPMPC_LIB=$L timeout -k 10 300 python3 -u bench.py $C4 $A > $OUT/c4_${V}_$r.json 2>> $OUT/bench.err
[ $r = 1 ] && GPMPC_LIB=$L timeout -k 10 300 python3 -u bench.py $C5 $A > $OUT/c5_${V}.json 2>> $OUT/bench.err
done
done
python3 - <<'PY'
import json, glob
for f in sorted(glob.glob("gpurun_out/loveby4/c*.json")):
    d = json.loads([x for x in open(f) if x.startswith("{")][-1])
    rv = d.get("roofline_variance", {})
    print(f.split("/")[-1], round(d["value"]), {k: round(v, 4) for k, v in d["kernel_ms_per_step"].items()}, round(rv.get("achieved", 0), 1))
PY
