#!/bin/bash
# HISTORICAL (round 3/4): the library reads no environment variables since round 5, so the GPMPC_* settings
# below no longer take effect; rerun with bench.py --lin-cache / --order / --overlap / --var-split / --waves.
# Round-4 A/B: overlapped step (cost-ranked halves, the second half's variance + SQP launches on a
# side stream) vs one variance launch then one SQP launch (GPMPC_OVERLAP=0), configs 3 / 4 / 5.
# bash tools/ab_overlap.sh OUTDIR
O=${1:?outdir}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 2
mkdir -p $O
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread \
    tests/test_gpu_semantics.py tests/test_gpu_parity.py tests/test_gpu_fullsize.py tests/test_gpu_love.py > $O/pytest.log 2>&1 || exit $?
A="--steps 20 --warmup 5 --no-cpu-baseline"
C4="--n-train 1000 --batch 1024"
C5="--model quad3d --n-train 4000 --fitc 2000 --horizon 40 --batch 512 --var-inputs dynamics"
for rep in 1 2; do
  for v in 1 0; do
    GPMPC_OVERLAP=$v timeout -k 10 200 python3 -u bench.py $A >> $O/c3_$v.jsonl 2>> $O/err || exit $?
    GPMPC_OVERLAP=$v timeout -k 10 300 python3 -u bench.py $A $C4 >> $O/c4_$v.jsonl 2>> $O/err || exit $?
    GPMPC_OVERLAP=$v timeout -k 10 400 python3 -u bench.py --steps 10 --warmup 3 --no-cpu-baseline $C5 >> $O/c5_$v.jsonl 2>> $O/err || exit $?
  done
done
python3 - $O <<'PY'
import json, sys
o = sys.argv[1]
for case in ("c3", "c4", "c5"):
    for v in ("1", "0"):
        ds = [json.loads(x) for x in open(f"{o}/{case}_{v}.jsonl") if x.startswith("{")]
        print(case, "overlap" if v == "1" else "sequential", " ".join(
            f"{d['value']:.0f} steps/s {d['ms_per_step']:.4f} ms (sqp {d['kernel_ms_per_step']['sqp']:.4f} var {d['kernel_ms_per_step']['variance']:.4f})" for d in ds),
            "status", ds[-1]["status_counts"])
PY
