#!/bin/bash
# Round-4 A/B: the hybrid (4x4x4_4b) Riccati factorisation against the 16x16x4 one, and the QP
# tolerance.  bash tools/ab_r4_ric.sh OUTDIR
O=${1:?outdir}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 2
mkdir -p $O
timeout -k 10 120 ./tools/ric_micro > $O/ric_micro.txt 2>&1 || exit $?
L=gp-mpc_amd/gpmpc/lib
# ric16: 16x16x4 factorisation, no helper overlap (round 3); hy: hybrid factorisation; prod: hybrid +
# helper overlap (the product library)
for v in prod hy ric16 prod hy ric16; do
  lib=$L/libgpmpc_mi355x.so; [ $v != prod ] && lib=$L/libgpmpc_mi355x_$v.so
  GPMPC_LIB=$PWD/$lib timeout -k 10 200 python3 -u bench.py --steps 20 --warmup 5 --no-cpu-baseline > $O/b_$v.json 2> $O/b_$v.err || exit $?
  cat $O/b_$v.json >> $O/all.jsonl
  GPMPC_LIB=$PWD/$lib timeout -k 10 200 python3 -u bench.py --steps 20 --warmup 5 --batch 128 --no-cpu-baseline > $O/b128_$v.json 2> $O/b128_$v.err || exit $?
  cat $O/b128_$v.json >> $O/all128.jsonl
done
for t in 1e-6 1e-7; do
  timeout -k 10 200 python3 -u bench.py --steps 20 --warmup 5 --qp-tol $t --no-cpu-baseline > $O/b_qp$t.json 2> $O/b_qp$t.err || exit $?
done
