#!/bin/bash
# gp_post_kernel with whole-panel staging and an unconditional K loop (FULL) against the previous
# library (base): the parity tests that reach it (predict at N = 1000, exact-variance closed loops,
# full-size config 5), then configs 4 and 5 with --variance exact (round 3).
set -e
OUT=gpurun_out/postfull
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p $OUT
LIB=$PWD/gp-mpc_amd/gpmpc/lib
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullsize.py -x -q --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -40 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
A="--steps 20 --warmup 5 --no-cpu-baseline --variance exact"
C4="--n-train 1000"
C5="--model quad3d --n-train 4000 --fitc 2000 --horizon 40 --batch 512 --var-inputs dynamics"
for V in new base; do
L=$LIB/libgpmpc_mi355x.so; [ $V != new ] && L=$LIB/libgpmpc_mi355x_$V.so
GPMPC_LIB=$L timeout -k 10 300 python3 -u bench.py $C4 $A > $OUT/c4x_$V.json 2>> $OUT/bench.err
GPMPC_LIB=$L timeout -k 10 400 python3 -u bench.py $C5 $A > $OUT/c5x_$V.json 2>> $OUT/bench.err
done
python3 - <<'PY'
import json, glob
for f in sorted(glob.glob("gpurun_out/postfull/c*.json")):
    d = json.loads([x for x in open(f) if x.startswith("{")][-1])
    rv = d.get("roofline_variance", {})
    print(f.split("/")[-1], round(d["value"]), {k: round(v, 4) for k, v in d["kernel_ms_per_step"].items()}, round(rv.get("achieved", 0), 1), d["status_counts"]["0"])
PY
