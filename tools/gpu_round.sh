#!/bin/bash
# One GPU verification pass that reports every failing test (run through gpurun from the repo root):
#   bash tools/gpu_round.sh OUTDIR [bench args...]
# 1. tools/status_census.py  2. pytest -m gpu (no -x: every failure is listed)  3. smoke  4. bench.py
# Each GPU step has its own time limit.  pytest's "tests failed" (exit 1) does not stop the pass;
# any other non-zero exit (crash, abort, time limit) ends it there.
OUT=${1:?outdir}
shift
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 2
mkdir -p "$OUT"
timeout -k 10 300 python3 -u tools/status_census.py > "$OUT/census.jsonl" 2> "$OUT/census.err" || exit $?
timeout -k 10 1000 python3 -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread \
    > "$OUT/pytest_gpu.log" 2>&1
rc=$?
tail -3 "$OUT/pytest_gpu.log"
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 180 python3 -u -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1 || exit $?
timeout -k 10 300 python3 -u bench.py "$@" > "$OUT/bench.json" 2> "$OUT/bench.err" || exit $?
cat "$OUT/bench.json"
exit $rc
