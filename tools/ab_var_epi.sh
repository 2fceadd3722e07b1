#!/bin/bash
# Next-step variance in the SQP epilogue (round 3): bit-exactness test, then the driver's config-3
# command with it on (share left to the next launch 1/16, 1/8, 1/4) and off (GPMPC_VAR_EPI=0).
set -e
OUT=gpurun_out/varepi
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p $OUT
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_launch.py -x -v --timeout 200 --timeout-method thread -k "epilogue or ordered" > $OUT/pytest.log 2>&1 || { tail -40 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
A="--steps 20 --warmup 5 --no-cpu-baseline"
for r in 1 2; do
GPMPC_VAR_EPI=0 timeout -k 10 200 python3 -u bench.py $A > $OUT/c3_off_$r.json 2>> $OUT/err
for F in 0.0625 0.125 0.25; do
GPMPC_VAR_EPI_FRAC=$F timeout -k 10 200 python3 -u bench.py $A > $OUT/c3_f${F}_$r.json 2>> $OUT/err
done
done
python3 - <<'PY'
import json, glob
for f in sorted(glob.glob("gpurun_out/varepi/c*.json")):
    d = json.loads([x for x in open(f) if x.startswith("{")][-1])
    print(f.split("/")[-1], round(d["value"]), {k: round(v, 4) for k, v in d["kernel_ms_per_step"].items()}, round(d["ms_per_step"], 4), d["status_counts"]["0"], d["sqp_kernel_ms_per_step_distribution"]["p50"])
PY
