#!/bin/bash
# HISTORICAL (round 3/4): the library reads no environment variables since round 5, so the GPMPC_* settings
# below no longer take effect; rerun with bench.py --lin-cache / --order / --overlap / --var-split / --waves.
# Round-4 A/B: (a) every launch ranked by cost (GPMPC_ORDER=2: the dispatcher then deals each cost
# quartile across the CUs) vs instance order for launches the device holds at once (configs 3, 4);
# (b) overlapped halves on/off for the multi-round config 5.  bash tools/ab_order.sh OUTDIR
O=${1:?outdir}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 2
mkdir -p $O
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread \
    tests/test_gpu_semantics.py tests/test_gpu_parity.py tests/test_gpu_launch.py > $O/pytest.log 2>&1 || exit $?
A="--steps 20 --warmup 5 --no-cpu-baseline"
C4="--n-train 1000 --batch 1024"
C5="--model quad3d --n-train 4000 --fitc 2000 --horizon 40 --batch 512 --var-inputs dynamics"
for rep in 1 2; do
  for v in 2 1; do
    GPMPC_ORDER=$v timeout -k 10 200 python3 -u bench.py $A >> $O/c3_o$v.jsonl 2>> $O/err || exit $?
    GPMPC_ORDER=$v timeout -k 10 300 python3 -u bench.py $A $C4 >> $O/c4_o$v.jsonl 2>> $O/err || exit $?
  done
  for v in 1 0; do
    GPMPC_OVERLAP=$v timeout -k 10 400 python3 -u bench.py --steps 10 --warmup 3 --no-cpu-baseline $C5 >> $O/c5_v$v.jsonl 2>> $O/err || exit $?
  done
done
python3 - $O <<'PY'
import json, sys
o = sys.argv[1]
for case, vs in (("c3", ("o2", "o1")), ("c4", ("o2", "o1")), ("c5", ("v1", "v0"))):
    for v in vs:
        ds = [json.loads(x) for x in open(f"{o}/{case}_{v}.jsonl") if x.startswith("{")]
        print(case, v, " ".join(
            f"{d['ms_per_step']:.4f} ms (sqp {d['kernel_ms_per_step']['sqp']:.4f} var {d['kernel_ms_per_step']['variance']:.4f})" for d in ds),
            "status", ds[-1]["status_counts"])
PY
