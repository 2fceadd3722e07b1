#!/bin/bash
# HISTORICAL (round 3/4): the library reads no environment variables since round 5, so the GPMPC_* settings
# below no longer take effect; rerun with bench.py --lin-cache / --order / --overlap / --var-split / --waves.
# Round-4 A/B: tightening variance with the column tiles split over 2 / 4 waves (gp_var_split_kernel,
# the automatic choice at few points) vs one wave per point tile (GPMPC_VAR_SPLIT=1).  Run on the build
# that still had the two-wave variant (GPMPC_VAR_SPLIT=2); the product keeps 1 and 4.
# bash tools/ab_varsplit.sh OUTDIR
O=${1:?outdir}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 2
mkdir -p $O
timeout -k 10 400 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread \
    tests/test_gpu_parity.py tests/test_gpu_golden.py tests/test_gpu_launch.py > $O/pytest.log 2>&1 || exit $?
A="--steps 20 --warmup 5 --no-cpu-baseline"
for rep in 1 2; do
  for v in auto 1 2 4; do
    for c in s8:--shard=0/8 s4:--shard=0/4 s2:--shard=0/2 s1:--shard=0/1; do
      n=${c%%:*}; a=${c#*:}
      GPMPC_VAR_SPLIT=$v timeout -k 10 200 python3 -u bench.py $A $a >> $O/${n}_$v.jsonl 2>> $O/err || exit $?
    done
    GPMPC_VAR_SPLIT=$v timeout -k 10 200 python3 -u bench.py $A --model cartpole --n-train 50 --horizon 20 --batch 256 \
        >> $O/c2_$v.jsonl 2>> $O/err || exit $?
  done
done
python3 - $O <<'PY'
import json, sys
o = sys.argv[1]
for case in ("s8", "s4", "s2", "s1", "c2"):
    for v in ("auto", "1", "2", "4"):
        ds = [json.loads(x) for x in open(f"{o}/{case}_{v}.jsonl") if x.startswith("{")]
        print(case, v, " ".join(f"{d['ms_per_step']:.4f} (sqp {d['kernel_ms_per_step']['sqp']:.4f} var {d['kernel_ms_per_step']['variance']:.4f})" for d in ds))
PY
