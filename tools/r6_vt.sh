#!/bin/bash
# Round-6: the next step's variances inside the SQP launch (GPMPC_TUNE_VAR_TAIL): its bit-exactness test and
# the launch / variance tests, the in-kernel variance's own time (GPMPC_VT_PROBE variant), then the driver's
# command at var_tail 0 / -1 (K = 256) / 128 / 384, twice.
# bash tools/r6_vt.sh OUTDIR
OUT=${1:?outdir}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 2
mkdir -p "$OUT"
timeout -k 10 600 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_launch.py \
    tests/test_gpu_semantics.py -m gpu -k "variance or tail or segments_follow" > "$OUT/pytest_vt.log" 2>&1 \
    || { tail -40 "$OUT/pytest_vt.log"; exit 1; }
tail -2 "$OUT/pytest_vt.log"
summ() { python3 -c "
import json,sys; d=json.load(open(sys.argv[1]))
k=d['kernel_ms_per_step'] or {}; l=d['roofline']['latency']
print(sys.argv[2], 'value %.0f' % d['value'], 'step ms %.4f' % d['ms_per_step'], 'sqp ms %.4f' % k.get('sqp', float('nan')), 'var ms %.4f' % k.get('variance', float('nan')), 'slowest %.4f mean %.4f' % (l['slowest_instance_ms_per_step'], l['mean_instance_ms_per_step']), 'status0', d['status_counts']['0'], 'late', d['launch'].get('var_tail_late'))" "$@"; }
GPMPC_LIB=$PWD/gp-mpc_amd/gpmpc/lib/libgpmpc_mi355x_vtp.so timeout -k 10 300 python3 -u bench.py --gpus 1 --steps 20 \
    --warmup 5 --no-cpu-baseline --no-single-instance --var-tail -1 > "$OUT/probe.json" 2> "$OUT/probe.err" || exit $?
python3 -c "
import json; d=json.load(open('$OUT/probe.json'))
print('probe: in-kernel variance us per computing instance %.1f' % (d['linearisations_per_step'] / 0.75 / 100))"
for r in 1 2; do
  for k in 0 -1 128 384; do
    timeout -k 10 300 python3 -u bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline --no-single-instance --var-tail $k \
        > "$OUT/vt${k}_r$r.json" 2> "$OUT/vt${k}_r$r.err" || exit $?
    summ "$OUT/vt${k}_r$r.json" "var_tail $k r$r"
  done
done
