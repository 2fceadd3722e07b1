#!/bin/bash
# Round-6 end-of-round evidence, part 2: the all-rank shard sweep (strong-scaling projection)
# and the packing analysis of config 5's two-round SQP launch (tools/packing.py).  bash tools/r6_final2.sh OUTDIR
set -e
OUT=${1:?outdir}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p "$OUT"
timeout -k 10 300 python3 -u tools/packing.py > "$OUT/packing_c5.txt" 2> "$OUT/packing_c5.err"
tail -2 "$OUT/packing_c5.txt" | head -1
bash tools/shard_sweep.sh "$OUT/shards_all" > "$OUT/shards_all_summary.txt" 2>&1
cat "$OUT/shards_all_summary.txt"
