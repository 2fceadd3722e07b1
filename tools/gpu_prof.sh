#!/bin/bash
# Round profile of the headline bench on one MI355X (run through gpurun from the repo root):
#   bash tools/gpu_prof.sh OUTDIR [bench args...]
# 1. rocprofv3 --kernel-trace --stats   (per-kernel durations; the last STEPS dispatches = timed region)
# 2. rocprofv3 --pmc FETCH_SIZE         (own pass, MI355X_MICROARCH.md: TCC counters one per pass)
# 3. rocprofv3 --pmc WRITE_SIZE         (own pass)
# 4. tools/pmc_summary.py -> OUTDIR/pmc_summary.json
# Every GPU step has its own time limit; the script stops at the first failure.
set -e
OUT=${1:?outdir}
shift
STEPS=40
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p "$OUT"
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace" -o run -- \
    python3 bench.py --steps $STEPS --warmup 20 --no-cpu-baseline "$@" > "$OUT/trace.log" 2>&1
timeout -k 10 400 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d "$OUT/fetch" -o run -- \
    python3 bench.py --steps $STEPS --warmup 20 --no-cpu-baseline "$@" > "$OUT/fetch.log" 2>&1
timeout -k 10 400 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d "$OUT/write" -o run -- \
    python3 bench.py --steps $STEPS --warmup 20 --no-cpu-baseline "$@" > "$OUT/write.log" 2>&1
WL=$(python3 -c "import json; l=[x for x in open('$OUT/trace.log') if x.startswith('{\"metric\"')][-1]; print(json.dumps({'workload': json.loads(l)['config']['workload']}))")
python3 tools/pmc_summary.py --trace "$OUT/trace" --fetch "$OUT/fetch" --write "$OUT/write" --last $STEPS \
    --config "$WL" -o "$OUT/pmc_summary.json"
