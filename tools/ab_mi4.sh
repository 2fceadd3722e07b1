#!/bin/bash
# HISTORICAL (round 3/4): the library reads no environment variables since round 5, so the GPMPC_* settings
# below no longer take effect; rerun with bench.py --lin-cache / --order / --overlap / --var-split / --waves.
# Round-4 A/B: one-wave SQP launches as four instances per workgroup (GPMPC_MI4) x overlapped
# halves (GPMPC_OVERLAP), configs 3 / 4 / 5.  bash tools/ab_mi4.sh OUTDIR
O=${1:?outdir}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 2
mkdir -p $O
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread \
    tests/test_gpu_semantics.py tests/test_gpu_parity.py tests/test_gpu_launch.py > $O/pytest.log 2>&1 || exit $?
A="--steps 20 --warmup 5 --no-cpu-baseline"
C4="--n-train 1000 --batch 1024"
for rep in 1 2; do
  for v in 11 10 01 00; do
    m=${v:0:1}; o=${v:1:1}
    GPMPC_MI4=$m GPMPC_OVERLAP=$o timeout -k 10 200 python3 -u bench.py $A >> $O/c3_$v.jsonl 2>> $O/err || exit $?
    GPMPC_MI4=$m GPMPC_OVERLAP=$o timeout -k 10 300 python3 -u bench.py $A $C4 >> $O/c4_$v.jsonl 2>> $O/err || exit $?
  done
done
python3 - $O <<'PY'
import json, sys
o = sys.argv[1]
for case in ("c3", "c4"):
    for v in ("11", "10", "01", "00"):
        ds = [json.loads(x) for x in open(f"{o}/{case}_{v}.jsonl") if x.startswith("{")]
        print(case, f"mi4={v[0]} overlap={v[1]}", " ".join(
            f"{d['ms_per_step']:.4f} ms (sqp {d['kernel_ms_per_step']['sqp']:.4f} var {d['kernel_ms_per_step']['variance']:.4f})" for d in ds))
PY
