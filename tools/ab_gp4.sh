#!/bin/bash
# GP tile sums entirely on v_mfma_f64_4x4x4_4b (exponents by z-block-rotated operands;
# round 3) against the 16x16x4 exponent variant (gp16): the parity tests that reach the GP sums, then
# configs 3 / 4 / 5 twice each.
set -e
OUT=gpurun_out/gp4
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p $OUT
LIB=$PWD/gp-mpc_amd/gpmpc/lib
GPMPC_LIB=$LIB/libgpmpc_mi355x_ne1.so timeout -k 10 500 python3 -u -m pytest tests/test_gpu_parity.py tests/test_gpu_golden.py tests/test_gpu_semantics.py tests/test_gpu_launch.py -x -q --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -40 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
A="--steps 20 --warmup 5 --no-cpu-baseline"
C4="--n-train 1000"
C5="--model quad3d --n-train 4000 --fitc 2000 --horizon 40 --batch 512 --var-inputs dynamics"
rm -f $OUT/c*.json
for r in 1 2; do
for V in ne1 new gp16; do
L=$LIB/libgpmpc_mi355x.so; [ $V != new ] && L=$LIB/libgpmpc_mi355x_$V.so
GPMPC_LIB=$L timeout -k 10 200 python3 -u bench.py $A > $OUT/c3_${V}_$r.json 2>> $OUT/err
GPMPC_LIB=$L timeout -k 10 300 python3 -u bench.py $C4 $A > $OUT/c4_${V}_$r.json 2>> $OUT/err
[ $r = 1 ] && GPMPC_LIB=$L timeout -k 10 300 python3 -u bench.py $C5 $A > $OUT/c5_${V}.json 2>> $OUT/err
[ $r = 1 ] && GPMPC_LIB=$L timeout -k 10 300 python3 -u bench.py --model cartpole --n-train 50 --horizon 20 --batch 256 $A > $OUT/c2_${V}.json 2>> $OUT/err
done
done
python3 - <<'PY'
import json, glob
for f in sorted(glob.glob("gpurun_out/gp4/c*.json")):
    d = json.loads([x for x in open(f) if x.startswith("{")][-1])
    print(f.split("/")[-1], round(d["value"]), {k: round(v, 4) for k, v in d["kernel_ms_per_step"].items()}, round(d["sqp_iter_mean"], 4), d["status_counts"]["0"])
PY
