#!/bin/bash
# Round-6 per-phase cycles of the slowest instance (timing build) at B = 1024 with the one-wave segment
# solve on and off: bash tools/r6_phase.sh OUTDIR
OUT=${1:?outdir}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 2
mkdir -p "$OUT"
for seg in 0 1; do
  timeout -k 10 150 python3 -u tools/phase_timing.py --batch 1024 --warmup 5 --steps 20 --seg $seg > "$OUT/phase_b1024_seg$seg.txt" 2>&1 || exit $?
done
tail -25 "$OUT"/phase_b1024_seg*.txt
