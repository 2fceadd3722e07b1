#!/bin/bash
# Round-6 per-phase cycles (timing build, tools/phase_timing.py) of the final kernel: the driver's B = 1024,
# the 8-GPU shard's 128 instances and config 5.  bash tools/r6_phase_final.sh OUTDIR
OUT=${1:?outdir}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 2
mkdir -p "$OUT"
timeout -k 10 200 python3 -u tools/phase_timing.py --batch 1024 --warmup 5 --steps 20 > "$OUT/phase_b1024.txt" 2>&1 || exit $?
timeout -k 10 200 python3 -u tools/phase_timing.py --batch 128 --warmup 5 --steps 20 > "$OUT/phase_b128.txt" 2>&1 || exit $?
timeout -k 10 300 python3 -u tools/phase_timing.py --model quad3d --batch 512 --n-train 4000 --fitc 2000 --horizon 40 \
    --var-inputs dynamics --warmup 5 --steps 20 > "$OUT/phase_config5.txt" 2>&1 || exit $?
tail -n 16 "$OUT"/phase_b1024.txt "$OUT"/phase_b128.txt
