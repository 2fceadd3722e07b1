#!/bin/bash
# Round-6: the tail boost (GPMPC_TUNE_TAIL) on the driver's command (B = 1024, one wave per instance):
# its parity test, then the bench line at K = 0 / 16 / 64 / 128 / 256, twice.  bash tools/r6_tail.sh OUTDIR
OUT=${1:?outdir}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 2
mkdir -p "$OUT"
timeout -k 10 600 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_launch.py -m gpu \
    -k "tail or segments_follow" > "$OUT/pytest_tail.log" 2>&1 || { tail -30 "$OUT/pytest_tail.log"; exit 1; }
tail -3 "$OUT/pytest_tail.log"
summ() { python3 -c "
import json,sys; d=json.load(open(sys.argv[1]))
k=d['kernel_ms_per_step'] or {}; l=d['roofline']['latency']
print(sys.argv[2], 'value %.0f' % d['value'], 'sqp ms %.4f' % k.get('sqp', float('nan')), 'slowest %.4f mean %.4f' % (l['slowest_instance_ms_per_step'], l['mean_instance_ms_per_step']), 'status0', d['status_counts']['0'], 'sqp_iter %.4f' % d['sqp_iter_mean'], 'tail_boost', d.get('launch', {}).get('tail_boost'))" "$@"; }
for r in 1 2; do
  for k in 0 16 64 128 256; do
    timeout -k 10 300 python3 -u bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline --no-single-instance --tail $k \
        > "$OUT/tail${k}_r$r.json" 2> "$OUT/tail${k}_r$r.err" || exit $?
    summ "$OUT/tail${k}_r$r.json" "tail $k r$r"
  done
done
