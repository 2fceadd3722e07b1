#!/bin/bash
# rocprofv3 kernel trace + stats of the secondary BASELINE configs at the driver's step counts
# (run through gpurun from the repo root):  bash tools/configs_prof.sh OUTDIR
set -e
OUT=${1:?outdir}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p "$OUT"
A="--steps 20 --warmup 5 --no-cpu-baseline"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/c2" -o run -- \
    python3 bench.py --model cartpole --n-train 50 --horizon 20 --batch 256 $A > "$OUT/c2.log" 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/c4" -o run -- \
    python3 bench.py --n-train 1000 $A > "$OUT/c4.log" 2>&1
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/c5" -o run -- \
    python3 bench.py --model quad3d --n-train 4000 --fitc 2000 --horizon 40 --batch 512 --var-inputs dynamics $A \
    > "$OUT/c5.log" 2>&1
