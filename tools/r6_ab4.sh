#!/bin/bash
# Round-6: round 5's kernel (r5k) on the metric's workload and shards (completes tools/r6_ab2.sh), then the
# configs A/B of tools/r6_ab3.sh.  bash tools/r6_ab4.sh OUTDIR
OUT=${1:?outdir}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 2
mkdir -p "$OUT"
summ() { python3 -c "
import json,sys; d=json.load(open(sys.argv[1]))
k=d['kernel_ms_per_step'] or {}
print(sys.argv[2], 'value %.0f' % d['value'], 'sqp ms %.4f' % k.get('sqp', float('nan')), 'var ms %.4f' % k.get('variance', float('nan')), 'status0', d['status_counts']['0'], 'sqp_iter %.4f' % d['sqp_iter_mean'])" "$@"; }
LIBDIR=$PWD/gp-mpc_amd/gpmpc/lib
for v in r5k product; do
  if [ $v = product ]; then unset GPMPC_LIB; else export GPMPC_LIB=$LIBDIR/libgpmpc_mi355x_$v.so; fi
  for sh in "" "--shard 0/2" "--shard 0/4" "--shard 0/8"; do
    tag=$v${sh:+_$(echo $sh | tr -d ' -/')}
    timeout -k 10 200 python3 -u bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline --no-single-instance $sh \
        > "$OUT/$tag.json" 2> "$OUT/$tag.err" || exit $?
    summ "$OUT/$tag.json" "$tag"
  done
done
unset GPMPC_LIB
bash tools/r6_ab3.sh "$OUT/configs"
