set -e
# HISTORICAL (round 3/4): the library reads no environment variables since round 5, so the GPMPC_* settings
# below no longer take effect; rerun with bench.py --lin-cache / --order / --overlap / --var-split / --waves.
OUT=gpurun_out/order2
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p $OUT
A="--steps 20 --warmup 5 --no-cpu-baseline"
C5="--model quad3d --n-train 4000 --fitc 2000 --horizon 40 --batch 512 --var-inputs dynamics"
timeout -k 10 300 python3 -u bench.py $C5 $A > $OUT/c5_order.json 2> $OUT/err
GPMPC_ORDER=0 timeout -k 10 300 python3 -u bench.py $C5 $A > $OUT/c5_noorder.json 2>> $OUT/err
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_launch.py -x -q --timeout 200 --timeout-method thread -k "ordered" > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
python3 - <<'PY'
import json
for f in ["c5_order", "c5_noorder"]:
    d = json.loads([x for x in open(f"gpurun_out/order2/{f}.json") if x.startswith("{")][-1])
    print(f, round(d["value"]), d["kernel_ms_per_step"], d["sqp_kernel_ms_per_step_distribution"]["per_step"][:8])
PY
