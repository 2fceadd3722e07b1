#!/bin/bash
# Round-6 same-box A/B of configs 4 and 5 (verdict item 5: the round-4 -> round-5 regressions; item 4: the
# sequential config-5 SQP kernel): this tree's library, round 5's sqp_kernel.hip (r5k) and round 4's (r4k),
# each with this tree's headers and C ABI.  bash tools/r6_ab3.sh OUTDIR
OUT=${1:?outdir}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 2
mkdir -p "$OUT"
summ() { python3 -c "
import json,sys; d=json.load(open(sys.argv[1]))
k=d['kernel_ms_per_step'] or {}
print(sys.argv[2], 'value %.0f' % d['value'], 'sqp ms %.4f' % k.get('sqp', float('nan')), 'var ms %.4f' % k.get('variance', float('nan')), 'status0', d['status_counts']['0'], 'sqp_iter %.4f' % d['sqp_iter_mean'])" "$@"; }
LIBDIR=$PWD/gp-mpc_amd/gpmpc/lib
C4="--n-train 1000 --batch 1024"
C5="--model quad3d --n-train 4000 --fitc 2000 --horizon 40 --batch 512 --var-inputs dynamics --overlap 0"
C2="--model cartpole --n-train 50 --horizon 20 --batch 256"
for v in product r5k r4k; do
  if [ $v = product ]; then unset GPMPC_LIB; else export GPMPC_LIB=$LIBDIR/libgpmpc_mi355x_$v.so; fi
  for c in c4 c5 c2; do
    case $c in c4) A=$C4;; c5) A=$C5;; c2) A=$C2;; esac
    timeout -k 10 300 python3 -u bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline --no-single-instance $A \
        > "$OUT/${v}_$c.json" 2> "$OUT/${v}_$c.err" || exit $?
    summ "$OUT/${v}_$c.json" "${v} $c"
  done
done
