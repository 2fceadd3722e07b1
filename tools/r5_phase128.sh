#!/bin/bash
# per-phase cycles of the slowest instance (timing build) at B=128, segment solve on / off
set -e
OUT=${1:?outdir}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p "$OUT"
for seg in 1 0; do
  timeout -k 10 120 python3 -u tools/phase_timing.py --batch 128 --warmup 5 --steps 20 --seg $seg > "$OUT/phase_b128_seg${seg}.txt" 2>&1
done
