#!/bin/bash
# Profile of the driver's own bench command (python3 bench.py --gpus 1 --steps 20 --warmup 5)
# on one MI355X, run through gpurun from the repo root:
#   bash tools/driver_prof.sh OUTDIR [extra bench args...]
# 1. the bench line itself (untraced)
# 2. rocprofv3 --kernel-trace --stats of the same command (per-dispatch durations)
# 3. one SQ PMC pass (wave cycles, wait/active split, VALU/MFMA issue) of the same command
# 4. FETCH_SIZE and WRITE_SIZE passes (each its own run) -> tools/pmc_summary.py
# Every GPU step has its own time limit; the script stops at the first failure.
set -e
OUT=${1:?outdir}
shift
ARGS="--gpus 1 --steps 20 --warmup 5"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p "$OUT"
timeout -k 10 300 python3 -u bench.py $ARGS "$@" > "$OUT/bench.json" 2> "$OUT/bench.err"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace" -o run -- \
    python3 bench.py $ARGS --no-cpu-baseline "$@" > "$OUT/trace.log" 2>&1
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY \
    SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_LDS --kernel-trace --output-format csv \
    -d "$OUT/sq" -o run -- python3 bench.py $ARGS --no-cpu-baseline "$@" > "$OUT/sq.log" 2>&1
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d "$OUT/fetch" -o run -- \
    python3 bench.py $ARGS --no-cpu-baseline "$@" > "$OUT/fetch.log" 2>&1
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d "$OUT/write" -o run -- \
    python3 bench.py $ARGS --no-cpu-baseline "$@" > "$OUT/write.log" 2>&1
WL=$(python3 -c "import json; l=[x for x in open('$OUT/trace.log') if x.startswith('{\"metric\"')][-1]; print(json.dumps({'workload': json.loads(l)['config']['workload']}))")
python3 tools/pmc_summary.py --trace "$OUT/trace" --fetch "$OUT/fetch" --write "$OUT/write" --last 20 \
    --config "$WL" -o "$OUT/pmc_summary.json"
cat "$OUT/bench.json"
