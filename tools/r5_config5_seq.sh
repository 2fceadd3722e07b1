#!/bin/bash
# Config 5 with the overlapped halves off (one variance launch, then one SQP launch of all 512
# instances): bench line and rocprofv3 kernel trace.  bash tools/r5_config5_seq.sh OUTDIR
set -e
OUT=${1:?outdir}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p "$OUT"
A="--model quad3d --n-train 4000 --fitc 2000 --horizon 40 --batch 512 --var-inputs dynamics --steps 20 --warmup 5 --no-cpu-baseline --no-single-instance --overlap 0"
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/c5seq" -o run -- \
    python3 bench.py $A > "$OUT/c5seq.log" 2>&1
