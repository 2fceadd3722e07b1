#!/bin/bash
# HISTORICAL (round 3/4): the library reads no environment variables since round 5, so the GPMPC_* settings
# below no longer take effect; rerun with bench.py --lin-cache / --order / --overlap / --var-split / --waves.
# Round-4 A/B: tightening variance split over 4 vs 8 waves per point tile (GPMPC_VAR_SPLIT=4/8) vs one
# (1) at the small shards, on the build that had the eight-wave variant (the product keeps 1 and 4).
# bash tools/ab_varsplit8.sh OUTDIR
O=${1:?outdir}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 2
mkdir -p $O
for v in 4 8; do
  GPMPC_VAR_SPLIT=$v timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread \
      tests/test_gpu_parity.py -k "tightening_variance" > $O/pytest_$v.log 2>&1 || exit $?
done
A="--steps 20 --warmup 5 --no-cpu-baseline"
for rep in 1 2; do
  for v in 1 4 8; do
    for c in s8:--shard=0/8 s4:--shard=0/4; do
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
for case in ("s8", "s4", "c2"):
    for v in ("1", "4", "8"):
        ds = [json.loads(x) for x in open(f"{o}/{case}_{v}.jsonl") if x.startswith("{")]
        print(case, v, " ".join(f"{d['ms_per_step']:.4f} (sqp {d['kernel_ms_per_step']['sqp']:.4f} var {d['kernel_ms_per_step']['variance']:.4f})" for d in ds))
PY
