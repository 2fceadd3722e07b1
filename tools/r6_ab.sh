#!/bin/bash
# Round-6 A/B pass (run through gpurun from the repo root): bash tools/r6_ab.sh OUTDIR
#  1. launch-shape parity tests (every wave count, segment solve on / off)
#  2. the driver's bench command (one wave per instance)
#  3. rank 0's strong-scaling shards (B = 128 / 256 / 512): this library (four waves: IPM split over
#     the waves) against the GPMPC_WSPL_SEG=0 variant (IPM on wave 0)
OUT=${1:?outdir}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 2
mkdir -p "$OUT"
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_launch.py -m gpu -v --timeout 200 --timeout-method thread > "$OUT/pytest_launch.log" 2>&1
rc=$?
tail -3 "$OUT/pytest_launch.log"
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
summ() { python3 -c "
import json,sys; d=json.load(open(sys.argv[1]))
k=d['kernel_ms_per_step'] or {}
print(sys.argv[2], 'value %.0f' % d['value'], 'sqp ms %.4f' % k.get('sqp', float('nan')), 'var ms %.4f' % k.get('variance', float('nan')), 'launch', d['launch']['waves'], d['launch']['segments'], 'status0', d['status_counts']['0'], 'sqp_iter %.4f' % d['sqp_iter_mean'])" "$@"; }
timeout -k 10 200 python3 -u bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline --no-single-instance \
    > "$OUT/b1024.json" 2> "$OUT/b1024.err" || exit $?
summ "$OUT/b1024.json" "B=1024"
for N in 8 4 2; do
  timeout -k 10 200 python3 -u bench.py --shard 0/$N --steps 20 --warmup 5 --no-cpu-baseline --no-single-instance \
      > "$OUT/shard0_$N.json" 2> "$OUT/shard0_$N.err" || exit $?
  summ "$OUT/shard0_$N.json" "shard 0/$N wspl"
  GPMPC_LIB=$PWD/gp-mpc_amd/gpmpc/lib/libgpmpc_mi355x_nowspl.so timeout -k 10 200 python3 -u bench.py --shard 0/$N --steps 20 \
      --warmup 5 --no-cpu-baseline --no-single-instance > "$OUT/shard0_${N}_nowspl.json" 2> "$OUT/shard0_${N}_nowspl.err" || exit $?
  summ "$OUT/shard0_${N}_nowspl.json" "shard 0/$N nowspl"
done
exit $rc
