#!/bin/bash
# Round-6: the forced segment fallback (GPMPC_TUNE_SEG_PIVOT = -1) against the one-segment recursion, the
# other segment tests, then rank 0's 4- and 8-GPU shards (the pivot threshold now a runtime value).
# bash tools/r6_fbtest.sh OUTDIR
OUT=${1:?outdir}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 2
mkdir -p "$OUT"
timeout -k 10 600 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_launch.py -m gpu \
    -k "segment or free_state or fallback" > "$OUT/pytest_fb.log" 2>&1 || { tail -30 "$OUT/pytest_fb.log"; exit 1; }
tail -3 "$OUT/pytest_fb.log"
for s in 0/4 0/8 0/4 0/8; do
  timeout -k 10 300 python3 -u bench.py --shard $s --steps 20 --warmup 5 --no-cpu-baseline --no-single-instance \
      > "$OUT/shard_${s/\//_}.json" 2> "$OUT/shard.err" || exit $?
  python3 -c "
import json; d=json.load(open('$OUT/shard_${s/\//_}.json')); print('shard $s', 'sqp %.4f' % d['kernel_ms_per_step']['sqp'])"
done
