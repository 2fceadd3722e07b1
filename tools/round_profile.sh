#!/bin/bash
# End-of-round evidence on one MI355X (run through gpurun from the repo root):
#   bash tools/round_profile.sh OUTDIR
# 1. bench.py (default N=1 line incl. the CPU baseline)   2. rocprofv3 kernel trace/stats + PMC passes
# 3. in-kernel phase breakdown (timing build)   4. the other BASELINE configs (one shard per GPU)
set -e
OUT=${1:?outdir}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p "$OUT"
timeout -k 10 240 python3 -u bench.py > "$OUT/bench.json" 2> "$OUT/bench.err"
bash tools/gpu_prof.sh "$OUT/prof"
timeout -k 10 120 python3 tools/phase_timing.py > "$OUT/phase_timing.txt" 2>&1
timeout -k 10 180 python3 -u bench.py --no-cpu-baseline --model cartpole --n-train 50 --horizon 20 --batch 256 > "$OUT/config2.json" 2>> "$OUT/bench.err"
timeout -k 10 180 python3 -u bench.py --no-cpu-baseline --n-train 1000 > "$OUT/config4.json" 2>> "$OUT/bench.err"
timeout -k 10 300 python3 -u bench.py --no-cpu-baseline --model quad3d --n-train 4000 --fitc 2000 --horizon 40 --batch 512 \
    --var-inputs dynamics --steps 30 --warmup 5 > "$OUT/config5.json" 2>> "$OUT/bench.err"
