#!/bin/bash
# Linearisation cache on/off at the driver's command (run through gpurun from the repo root):
#   bash tools/lin_ab.sh OUTDIR [bench args...]
set -e
OUT=${1:?outdir}; shift
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p "$OUT"
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_semantics.py -x -v --timeout 120 --timeout-method thread \
    > "$OUT/pytest_sem.log" 2>&1
for rep in 1 2; do
  GPMPC_LIN_CACHE=0 timeout -k 10 120 python3 bench.py --no-cpu-baseline "$@" > "$OUT/bench_off_$rep.json" 2> "$OUT/bench_off_$rep.err"
  timeout -k 10 120 python3 bench.py --no-cpu-baseline "$@" > "$OUT/bench_on_$rep.json" 2> "$OUT/bench_on_$rep.err"
done
python3 - "$OUT" <<'PY'
import json, sys, glob
for f in sorted(glob.glob(sys.argv[1] + "/bench_*.json")):
    d = json.loads([x for x in open(f) if x.startswith("{")][-1])
    print(f.split("/")[-1], f"value {d['value']:.0f} sqp {d['kernel_ms_per_step']['sqp']:.4f} ms var {d['kernel_ms_per_step']['variance']:.4f} sqp_iter {d['sqp_iter_mean']:.3f} max {d.get('sqp_iter_max')} status {d['status_counts']}")
PY
