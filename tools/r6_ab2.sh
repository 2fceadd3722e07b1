#!/bin/bash
# Round-6 A/B of the SQP-kernel variants on the metric's workload (run through gpurun from the repo root):
#   bash tools/r6_ab2.sh OUTDIR
# libraries: this tree's (phase_lane on the one-wave and quad3d kernels), pl0 (phase_lane off), pl2 (on every
# kernel), r5k (round 5's sqp_kernel.hip with this tree's headers and C ABI); for each: B = 1024 and rank 0's
# 2-, 4-, 8-GPU shards of the metric's batch, --steps 20 --warmup 5.
OUT=${1:?outdir}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 2
mkdir -p "$OUT"
summ() { python3 -c "
import json,sys; d=json.load(open(sys.argv[1]))
k=d['kernel_ms_per_step'] or {}
print(sys.argv[2], 'value %.0f' % d['value'], 'sqp ms %.4f' % k.get('sqp', float('nan')), 'var ms %.4f' % k.get('variance', float('nan')), 'launch', d['launch']['waves'], d['launch']['segments'], 'status0', d['status_counts']['0'], 'sqp_iter %.4f' % d['sqp_iter_mean'])" "$@"; }
LIBDIR=$PWD/gp-mpc_amd/gpmpc/lib
for v in product pl0 pl2 r5k; do
  if [ $v = product ]; then unset GPMPC_LIB; else export GPMPC_LIB=$LIBDIR/libgpmpc_mi355x_$v.so; fi
  for sh in "" "--shard 0/2" "--shard 0/4" "--shard 0/8"; do
    tag=$v${sh:+_$(echo $sh | tr -d ' -/')}
    timeout -k 10 200 python3 -u bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline --no-single-instance $sh \
        > "$OUT/$tag.json" 2> "$OUT/$tag.err" || exit $?
    summ "$OUT/$tag.json" "$tag"
  done
done
