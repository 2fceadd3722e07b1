#!/bin/bash
# parity of every launch shape, the segment micro-benchmark, and the shard timings (seg on / off)
set -e
OUT=${1:?outdir}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p "$OUT"
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_launch.py -x -v --timeout 120 --timeout-method thread \
    -k "launch_shapes" > "$OUT/pytest_launch.log" 2>&1
timeout -k 10 120 ./tools/seg_micro > "$OUT/seg_micro.txt" 2>&1
timeout -k 10 120 ./tools/ric_micro > "$OUT/ric_micro.txt" 2>&1
for shard in 0/8 0/4 0/2; do
  for seg in 0 1; do
    n=$(echo $shard | tr / _)
    timeout -k 10 120 python3 -u bench.py --shard $shard --steps 20 --warmup 5 --seg $seg --no-cpu-baseline \
        > "$OUT/shard_${n}_seg${seg}.json" 2> "$OUT/shard_${n}_seg${seg}.err"
  done
done
grep -h '"ms_per_step"' "$OUT"/shard_*.json | python3 -c "
import sys, json
for l in sys.stdin:
    d = json.loads(l); print(d['config']['batch_per_gpu'], round(d['ms_per_step'], 4), d['kernel_ms_per_step'], d['status_counts'])"
