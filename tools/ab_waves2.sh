#!/bin/bash
# HISTORICAL (round 3/4): the library reads no environment variables since round 5, so the GPMPC_* settings
# below no longer take effect; rerun with bench.py --lin-cache / --order / --overlap / --var-split / --waves.
# Two waves per instance for batches of CUs < B <= 2 CUs (round 3): launch-shape parity, then the
# config-3 shard of 512 instances and config 2 at B = 512 with waves auto (2) / 1 / 4.
set -e
OUT=gpurun_out/waves2
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p $OUT
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_launch.py -x -q --timeout 200 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -40 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
A="--steps 20 --warmup 5 --no-cpu-baseline"
for W in 2 1; do
GPMPC_WAVES=$W timeout -k 10 200 python3 -u bench.py --batch 512 $A > $OUT/c3b512_w$W.json 2>> $OUT/err
GPMPC_WAVES=$W timeout -k 10 200 python3 -u bench.py --model cartpole --n-train 50 --horizon 20 --batch 512 $A > $OUT/c2b512_w$W.json 2>> $OUT/err
done
timeout -k 10 200 python3 -u bench.py --batch 512 $A > $OUT/c3b512_auto.json 2>> $OUT/err
python3 - <<'PY'
import json, glob
for f in sorted(glob.glob("gpurun_out/waves2/c*.json")):
    d = json.loads([x for x in open(f) if x.startswith("{")][-1])
    print(f.split("/")[-1], round(d["value"]), {k: round(v, 4) for k, v in d["kernel_ms_per_step"].items()}, round(d["ms_per_step"], 4), d["status_counts"]["0"])
PY
