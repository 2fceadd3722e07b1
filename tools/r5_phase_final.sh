#!/bin/bash
# per-phase cycles of the slowest instance (timing build): the 8-GPU shard (B=128, four waves, three
# segments), the 2-GPU shard (B=512, two waves, two segments) and the headline batch (B=1024, one wave)
set -e
OUT=${1:?outdir}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p "$OUT"
for B in 128 512 1024; do
  timeout -k 10 150 python3 -u tools/phase_timing.py --batch $B --warmup 5 --steps 20 > "$OUT/phase_b${B}.txt" 2>&1
done
