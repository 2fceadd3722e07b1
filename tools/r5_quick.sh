#!/bin/bash
# quick A/B loop: launch-shape parity, segment micro-benchmark, the strong-scaling shards (rank 0)
# and the headline batch (B=1024), SQP/variance kernel times.  bash tools/r5_quick.sh OUTDIR
set -e
OUT=${1:?outdir}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p "$OUT"
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_launch.py -x -v --timeout 120 --timeout-method thread \
    -k "launch_shapes" > "$OUT/pytest_launch.log" 2>&1
timeout -k 10 120 ./tools/seg_micro > "$OUT/seg_micro.txt" 2>&1
for shard in 0/1 0/2 0/4 0/8; do
  n=$(echo $shard | tr / _)
  timeout -k 10 120 python3 -u bench.py --shard $shard --steps 20 --warmup 5 --no-cpu-baseline --no-single-instance \
      > "$OUT/shard_${n}.json" 2> "$OUT/shard_${n}.err"
done
grep -h '"ms_per_step"' "$OUT"/shard_*.json | python3 -c "
import sys, json
for l in sys.stdin:
    d = json.loads(l); print(d['config']['batch_per_gpu'], round(d['ms_per_step'], 4), {k: round(v, 4) for k, v in d['kernel_ms_per_step'].items()}, d['status_counts'])"
