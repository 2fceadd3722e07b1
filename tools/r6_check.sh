#!/bin/bash
# Round-6 GPU verification pass (run through gpurun from the repo root):
#   bash tools/r6_check.sh OUTDIR [pytest -k expression]
# 1. pytest -m gpu (no -x: every failure is listed)  2. smoke()  3. the driver's bench command.
# Each GPU step has its own time limit; pytest's "tests failed" (exit 1) does not stop the pass,
# any other non-zero exit (crash, abort, time limit) ends it there.
OUT=${1:?outdir}
K=${2:-}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 2
mkdir -p "$OUT"
if [ -n "$K" ]; then
  timeout -k 10 900 python3 -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread -k "$K" \
      > "$OUT/pytest_gpu.log" 2>&1
else
  timeout -k 10 1000 python3 -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread \
      > "$OUT/pytest_gpu.log" 2>&1
fi
rc=$?
tail -3 "$OUT/pytest_gpu.log"
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 180 python3 -u -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1 || exit $?
timeout -k 10 300 python3 -u bench.py --gpus 1 --steps 20 --warmup 5 > "$OUT/bench.json" 2> "$OUT/bench.err" || exit $?
python3 -c "
import json; d=json.load(open('$OUT/bench.json'))
r=d['roofline']; print('value', d['value'], 'sqp ms', d['kernel_ms_per_step'], 'frac', r['frac'], 'latency', r['latency'], 'build', d['build'])"
exit $rc
