#!/bin/bash
# GPU tests + smoke + the round profile (tools/round_profile.sh) + config 5 with the linearisation
# cache off, on one MI355X (run through gpurun from the repo root):  bash tools/check_and_profile.sh OUTDIR
set -e
OUT=${1:?outdir}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p "$OUT"
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > "$OUT/pytest_gpu.log" 2>&1
timeout -k 10 180 python3 -u -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1
bash tools/round_profile.sh "$OUT"
GPMPC_LIN_CACHE=0 timeout -k 10 300 python3 -u bench.py --model quad3d --n-train 4000 --fitc 2000 --horizon 40 \
    --batch 512 --var-inputs dynamics --steps 20 --warmup 5 --no-cpu-baseline > "$OUT/config5_nocache.json" 2>> "$OUT/bench.err"
