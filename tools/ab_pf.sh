#!/bin/bash
# Round-4 A/B: sweep stage operands two stages ahead (product) vs one (pf1 variant), plus the
# recursion micro-benchmark.  bash tools/ab_pf.sh OUTDIR
O=${1:?outdir}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 2
mkdir -p $O
timeout -k 10 120 ./tools/ric_micro > $O/ric_micro.txt 2>&1 || exit $?
L=$PWD/gp-mpc_amd/gpmpc/lib
for v in prod pf1 prod pf1; do
  lib=$L/libgpmpc_mi355x.so; [ $v != prod ] && lib=$L/libgpmpc_mi355x_$v.so
  GPMPC_LIB=$lib timeout -k 10 200 python3 -u bench.py --steps 20 --warmup 5 --no-cpu-baseline >> $O/b_$v.jsonl 2>> $O/b_$v.err || exit $?
  GPMPC_LIB=$lib timeout -k 10 200 python3 -u bench.py --steps 20 --warmup 5 --batch 128 --no-cpu-baseline >> $O/b128_$v.jsonl 2>> $O/b128_$v.err || exit $?
done
