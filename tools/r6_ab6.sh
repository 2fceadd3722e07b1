#!/bin/bash
# Round-6: which of the round-6 additions costs the multi-wave shards their 3% against round 5 (nofb: no pivot check/fallback, nots: no solve stamp).  bash tools/r6_ab6.sh OUTDIR
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
for v in product nofb nots nofbts r5k product nofb nots nofbts r5k; do
  run $v shard04 --shard 0/4 || exit $?
  run $v shard08 --shard 0/8 || exit $?
done
