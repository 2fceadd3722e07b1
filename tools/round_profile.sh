#!/bin/bash
# End-of-round evidence on one MI355X (run through gpurun from the repo root):
#   bash tools/round_profile.sh OUTDIR
# 1. the driver's own command (bench.py --gpus 1 --steps 20 --warmup 5, with the CPU baseline),
#    rocprofv3 kernel trace/stats, one SQ PMC pass and the FETCH_SIZE / WRITE_SIZE passes of the
#    same command (tools/driver_prof.sh)
# 2. in-kernel phase breakdown (timing build) of configs 3 and 5
# 3. the other BASELINE configs (one shard per GPU), each with its CPU baseline (1 core, all cores);
#    configs 4 and 5 at the default (the reference's gpytorch fast_pred_var: LOVE above 800 rows) and
#    with --variance exact
set -e
OUT=${1:?outdir}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p "$OUT"
bash tools/driver_prof.sh "$OUT/driver"
timeout -k 10 120 python3 tools/phase_timing.py --warmup 5 > "$OUT/phase_timing.txt" 2>&1
timeout -k 10 300 python3 tools/phase_timing.py --model quad3d --n-train 4000 --fitc 2000 --horizon 40 --batch 512 \
    --var-inputs dynamics --warmup 3 --steps 3 > "$OUT/phase_timing_config5.txt" 2>&1
timeout -k 10 240 python3 -u bench.py --model cartpole --n-train 50 --horizon 20 --batch 256 \
    --steps 20 --warmup 5 > "$OUT/config2.json" 2>> "$OUT/bench.err"
timeout -k 10 300 python3 -u bench.py --n-train 1000 --batch 1024 --steps 20 --warmup 5 > "$OUT/config4.json" 2>> "$OUT/bench.err"
timeout -k 10 600 python3 -u bench.py --model quad3d --n-train 4000 --fitc 2000 --horizon 40 --batch 512 \
    --var-inputs dynamics --steps 20 --warmup 5 > "$OUT/config5.json" 2>> "$OUT/bench.err"
timeout -k 10 300 python3 -u bench.py --n-train 1000 --batch 1024 --steps 20 --warmup 5 --variance exact --no-cpu-baseline \
    > "$OUT/config4_exact.json" 2>> "$OUT/bench.err"
timeout -k 10 600 python3 -u bench.py --model quad3d --n-train 4000 --fitc 2000 --horizon 40 --batch 512 \
    --var-inputs dynamics --steps 20 --warmup 5 --variance exact --no-cpu-baseline > "$OUT/config5_exact.json" 2>> "$OUT/bench.err"
