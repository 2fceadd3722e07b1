#!/bin/bash
# Multi-rank bench rehearsal on a one-GPU box (run through gpurun): two ranks share GPU 0 over gloo
# (RCCL refuses two ranks on one GPU), launched as the driver launches the N > 1 legs.
set -e
OUT=${1:?outdir}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p "$OUT"
GPMPC_DIST_BACKEND=gloo timeout -k 10 300 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
    --master-addr 127.0.0.1 --master-port 29511 bench.py --gpus 2 --steps 5 --warmup 2 --no-cpu-baseline \
    > "$OUT/bench_2ranks.json" 2> "$OUT/bench_2ranks.err"
timeout -k 10 300 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 1 \
    --master-addr 127.0.0.1 --master-port 29512 bench.py --gpus 1 --steps 5 --warmup 2 --no-cpu-baseline \
    > "$OUT/bench_torchrun1.json" 2> "$OUT/bench_torchrun1.err"
tail -c 600 "$OUT/bench_2ranks.json"; echo; tail -c 300 "$OUT/bench_torchrun1.json"
