#!/bin/bash
# Round 5: per-phase cycles of the slowest instance (timing build) for the two-segment solve at the
# strong-scaling shards, and the lincache census print.  bash tools/r5_phase.sh OUTDIR
set -e
OUT=${1:?outdir}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p "$OUT"
for B in 128 256 512; do
  for seg in 0 1; do
    timeout -k 10 120 python3 -u tools/phase_timing.py --batch $B --warmup 5 --steps 20 --seg $seg > "$OUT/phase_b${B}_seg${seg}.txt" 2>&1
  done
done
timeout -k 10 200 python3 -u -m pytest tests/test_gpu_semantics.py -x -s -v --timeout 150 --timeout-method thread \
    -k "linearisation_cache and quad2d" > "$OUT/census_lincache.log" 2>&1
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_fullsize.py -x -s -v --timeout 250 --timeout-method thread \
    -k "shipped_defaults" > "$OUT/config3_defaults.log" 2>&1
