#!/bin/bash
# Branch-free LOVE kernel at two waves per SIMD (-DGPMPC_LOVE_W2, 256 VGPRs) against one (round 3).
set -e
OUT=gpurun_out/lovew2
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p $OUT
LIB=$PWD/gp-mpc_amd/gpmpc/lib
GPMPC_LIB=$LIB/libgpmpc_mi355x_lw2.so timeout -k 10 300 python3 -u -m pytest tests/test_gpu_love.py -x -q --timeout 200 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
A="--steps 20 --warmup 5 --no-cpu-baseline"
C5="--model quad3d --n-train 4000 --fitc 2000 --horizon 40 --batch 512 --var-inputs dynamics"
for r in 1 2; do
for V in new lw2; do
L=$LIB/libgpmpc_mi355x.so; [ $V != new ] && L=$LIB/libgpmpc_mi355x_$V.so
GPMPC_LIB=$L timeout -k 10 300 python3 -u bench.py --n-train 1000 $A > $OUT/c4_${V}_$r.json 2>> $OUT/err
[ $r = 1 ] && GPMPC_LIB=$L timeout -k 10 300 python3 -u bench.py $C5 $A > $OUT/c5_${V}.json 2>> $OUT/err
done
done
python3 - <<'PY'
import json, glob
for f in sorted(glob.glob("gpurun_out/lovew2/c*.json")):
    d = json.loads([x for x in open(f) if x.startswith("{")][-1])
    print(f.split("/")[-1], round(d["value"]), {k: round(v, 4) for k, v in d["kernel_ms_per_step"].items()})
PY
