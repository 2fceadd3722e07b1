#!/bin/bash
# One GPU verification pass (run through gpurun from the repo root):
#   bash tools/gpu_check.sh OUTDIR [bench args...]
# 1. pytest -m gpu (parity tests through the C ABI)  2. __graft_entry__.smoke()  3. bench.py (N=1)
# Every GPU step has its own time limit; the script stops at the first failure.
set -e
OUT=${1:?outdir}
shift
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p "$OUT"
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread \
    > "$OUT/pytest_gpu.log" 2>&1
timeout -k 10 180 python3 -u -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1
timeout -k 10 300 python3 -u bench.py "$@" > "$OUT/bench.json" 2> "$OUT/bench.err"
cat "$OUT/bench.json"
