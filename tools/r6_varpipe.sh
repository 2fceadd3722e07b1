#!/bin/bash
# Round-6: the variance kernel's next-panel kernel values under the current panel's MFMAs (GPMPC_VAR_PIPE)
# against the previous order (vp0): variance parity tests, then the driver's command and rank 0's 8-GPU
# shard, twice, with the variance kernel's HIP-event time.  bash tools/r6_varpipe.sh OUTDIR
OUT=${1:?outdir}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 2
mkdir -p "$OUT"
timeout -k 10 600 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_parity.py \
    tests/test_gpu_golden.py -m gpu -k "variance or tightening" > "$OUT/pytest_var.log" 2>&1 || { tail -30 "$OUT/pytest_var.log"; exit 1; }
tail -2 "$OUT/pytest_var.log"
summ() { python3 -c "
import json,sys; d=json.load(open(sys.argv[1]))
k=d['kernel_ms_per_step'] or {}
print(sys.argv[2], 'value %.0f' % d['value'], 'sqp ms %.4f' % k.get('sqp', float('nan')), 'var ms %.4f' % k.get('variance', float('nan')), 'var frac', d['roofline_variance']['frac'])" "$@"; }
LIBDIR=$PWD/gp-mpc_amd/gpmpc/lib
for r in 1 2; do
  for v in product vp0; do
    if [ $v = product ]; then unset GPMPC_LIB; else export GPMPC_LIB=$LIBDIR/libgpmpc_mi355x_$v.so; fi
    timeout -k 10 300 python3 -u bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline --no-single-instance \
        > "$OUT/${v}_r$r.json" 2> "$OUT/${v}_r$r.err" || exit $?
    summ "$OUT/${v}_r$r.json" "$v b1024 r$r"
    timeout -k 10 300 python3 -u bench.py --shard 0/8 --steps 20 --warmup 5 --no-cpu-baseline --no-single-instance \
        > "$OUT/${v}_s8_r$r.json" 2> "$OUT/${v}_s8_r$r.err" || exit $?
    summ "$OUT/${v}_s8_r$r.json" "$v shard08 r$r"
  done
done
