#!/bin/bash
# Round-6: the fallback posted by wave 0 as its own command (helpers never read the flag): segment tests (incl. the fallback case), then shards against nofb and round 5.  bash tools/r6_ab9.sh OUTDIR
OUT=${1:?outdir}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 2
mkdir -p "$OUT"
summ() { python3 -c "
import json,sys; d=json.load(open(sys.argv[1]))
k=d['kernel_ms_per_step'] or {}
print(sys.argv[2], 'value %.0f' % d['value'], 'sqp ms %.4f' % k.get('sqp', float('nan')), 'var ms %.4f' % k.get('variance', float('nan')), 'status0', d['status_counts']['0'], 'sqp_iter %.4f' % d['sqp_iter_mean'])" "$@"; }
LIBDIR=$PWD/gp-mpc_amd/gpmpc/lib
run() {   # lib tag args...
  local v=$1 tag=$2; shift 2
  if [ $v = product ]; then unset GPMPC_LIB; else export GPMPC_LIB=$LIBDIR/libgpmpc_mi355x_$v.so; fi
  timeout -k 10 300 python3 -u bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline --no-single-instance "$@" \
      > "$OUT/${v}_$tag.json" 2> "$OUT/${v}_$tag.err" || return $?
  summ "$OUT/${v}_$tag.json" "${v} $tag"
}
timeout -k 10 600 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_launch.py -m gpu -k "segment or free_state or launch_shapes" > "$OUT/pytest_seg.log" 2>&1 || { tail -30 "$OUT/pytest_seg.log"; exit 1; }
tail -3 "$OUT/pytest_seg.log"
for v in product nofb product nofb product nofb; do
  run $v shard04 --shard 0/4 || exit $?
  run $v shard08 --shard 0/8 || exit $?
done
