#!/bin/bash
# Phase breakdowns (timing build) of the launch shapes: config 3 stage-by-stage vs condensed,
# config 2 with one / four waves per instance, with and without condensing.
set -e
OUT=gpurun_out/r3d
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p $OUT
timeout -k 10 120 python3 tools/phase_timing.py --warmup 5 --no-condense --waves 1 > $OUT/c3_w1c0.txt 2>&1
timeout -k 10 120 python3 tools/phase_timing.py --warmup 5 --waves 1 > $OUT/c3_w1c1.txt 2>&1
for W in 1 4; do for C in 0 1; do
  NC=""; [ $C = 0 ] && NC="--no-condense"
  timeout -k 10 120 python3 tools/phase_timing.py --model cartpole --n-train 50 --horizon 20 --batch 256 --warmup 5 --waves $W $NC > $OUT/c2_w${W}c${C}.txt 2>&1
done; done
timeout -k 10 120 python3 tools/phase_timing.py --warmup 5 --batch 128 --waves 4 > $OUT/c3_b128_w4c1.txt 2>&1
timeout -k 10 120 python3 tools/phase_timing.py --warmup 5 --batch 128 --waves 1 --no-condense > $OUT/c3_b128_w1c0.txt 2>&1
cat $OUT/*.txt | grep -v amdgpu.ids
