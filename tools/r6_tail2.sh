#!/bin/bash
# Round-6: the tail boost where the batch leaves SIMDs free (2 CUs < B < 4 CUs): B = 768 and 896 at
# K = 0 / spare SIMDs / half of them, twice.  bash tools/r6_tail2.sh OUTDIR
OUT=${1:?outdir}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 2
mkdir -p "$OUT"
summ() { python3 -c "
import json,sys; d=json.load(open(sys.argv[1]))
k=d['kernel_ms_per_step'] or {}; l=d['roofline']['latency']
print(sys.argv[2], 'value %.0f' % d['value'], 'sqp ms %.4f' % k.get('sqp', float('nan')), 'slowest %.4f mean %.4f' % (l['slowest_instance_ms_per_step'], l['mean_instance_ms_per_step']), 'status0', d['status_counts']['0'], 'sqp_iter %.4f' % d['sqp_iter_mean'], 'tail_boost', d.get('launch', {}).get('tail_boost'))" "$@"; }
for r in 1 2; do
  for bk in 768:0 768:128 768:256 896:0 896:64 896:128; do
    b=${bk%%:*}; k=${bk##*:}
    timeout -k 10 300 python3 -u bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline --no-single-instance \
        --batch $b --tail $k > "$OUT/b${b}_tail${k}_r$r.json" 2> "$OUT/b${b}_tail${k}_r$r.err" || exit $?
    summ "$OUT/b${b}_tail${k}_r$r.json" "B $b tail $k r$r"
  done
done
