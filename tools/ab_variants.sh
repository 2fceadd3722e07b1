#!/bin/bash
# A/B of library variants on one GPU (run through gpurun from the repo root):
#   bash tools/ab_variants.sh OUTDIR name1 name2 ...   (gp-mpc_amd/gpmpc/lib/libgpmpc_mi355x_<name>{,_timing}.so)
# For each: bench.py (no CPU baseline) and tools/phase_timing.py; stops at the first failure.
set -e
OUT=${1:?outdir}; shift
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p "$OUT"
LIB=$GRAFT_REPO_ROOT/gp-mpc_amd/gpmpc/lib
for rep in 1 2; do
for v in "$@"; do
  GPMPC_LIB=$LIB/libgpmpc_mi355x_$v.so timeout -k 10 120 python3 bench.py --no-cpu-baseline $BENCH_ARGS \
      > "$OUT/bench_${v}_$rep.json" 2> "$OUT/bench_${v}_$rep.err"
done
done
for v in "$@"; do
  [ -f $LIB/libgpmpc_mi355x_${v}_timing.so ] || continue
  GPMPC_LIB=$LIB/libgpmpc_mi355x_${v}_timing.so timeout -k 10 120 python3 tools/phase_timing.py $PHASE_ARGS > "$OUT/phase_$v.txt" 2>&1
done
python3 - "$OUT" "$@" <<'PY'
import json, sys, glob
out = sys.argv[1]
for v in sys.argv[2:]:
    for f in sorted(glob.glob(f"{out}/bench_{v}_*.json")):
        l = [x for x in open(f) if x.startswith("{")][-1]
        d = json.loads(l)
        print(f"{v:8s} {f[-6:-5]} value {d['value']:.0f}  sqp {d['kernel_ms_per_step']['sqp']:.4f} ms  var {d['kernel_ms_per_step']['variance']:.4f} ms  sqp_iter {d['sqp_iter_mean']:.3f} status {d['status_counts']}")
PY
