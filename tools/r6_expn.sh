#!/bin/bash
# Round-6: the triangular variance kernel's four kernel values per panel through exp_rbf_n (vx1) against
# exp_rbf (product): the driver's command, three times each.  bash tools/r6_expn.sh OUTDIR
OUT=${1:?outdir}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 2
mkdir -p "$OUT"
LIBDIR=$PWD/gp-mpc_amd/gpmpc/lib
for r in 1 2 3; do
  for v in product vx1; do
    if [ $v = product ]; then unset GPMPC_LIB; else export GPMPC_LIB=$LIBDIR/libgpmpc_mi355x_$v.so; fi
    timeout -k 10 300 python3 -u bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline --no-single-instance \
        > "$OUT/${v}_r$r.json" 2> "$OUT/${v}_r$r.err" || exit $?
    python3 -c "
import json; d=json.load(open('$OUT/${v}_r$r.json')); k=d['kernel_ms_per_step']
print('$v r$r', 'value %.0f' % d['value'], 'sqp %.4f var %.4f' % (k['sqp'], k['variance']))"
  done
done
