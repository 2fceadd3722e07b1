#!/bin/bash
# Round-4 A/B: branch-free stores of non-storing lanes to one shared dummy slot (product) vs one slot
# per lane (libgpmpc_mi355x_prev.so): recursion micro-benchmark + LDS counters, GPU tests, benches.
# bash tools/ab_dummy.sh OUTDIR
O=${1:?outdir}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 2
mkdir -p $O
bash tools/ric_lds_pmc.sh $O/ric > $O/ric_pmc.txt 2>&1 || exit $?
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/ > $O/pytest.log 2>&1 || exit $?
L=$PWD/gp-mpc_amd/gpmpc/lib
A="--steps 20 --warmup 5 --no-cpu-baseline"
for v in prod prev prod prev; do
  lib=$L/libgpmpc_mi355x.so; [ $v != prod ] && lib=$L/libgpmpc_mi355x_$v.so
  GPMPC_LIB=$lib timeout -k 10 200 python3 -u bench.py $A >> $O/b_$v.jsonl 2>> $O/err || exit $?
  GPMPC_LIB=$lib timeout -k 10 200 python3 -u bench.py $A --shard 0/8 >> $O/s8_$v.jsonl 2>> $O/err || exit $?
  GPMPC_LIB=$lib timeout -k 10 200 python3 -u bench.py $A --model cartpole --n-train 50 --horizon 20 --batch 256 \
      >> $O/c2_$v.jsonl 2>> $O/err || exit $?
done
cat $O/ric/ric_micro.txt $O/ric_pmc.txt
python3 - $O <<'PY'
import json, sys
o = sys.argv[1]
for case in ("b", "s8", "c2"):
    for v in ("prod", "prev"):
        ds = [json.loads(x) for x in open(f"{o}/{case}_{v}.jsonl") if x.startswith("{")]
        print(case, v, " ".join(f"{d['ms_per_step']:.4f}/{d['kernel_ms_per_step']['sqp']:.4f}" for d in ds),
              "status", ds[-1]["status_counts"])
PY
