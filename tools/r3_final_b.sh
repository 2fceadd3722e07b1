#!/bin/bash
# Round-3 evidence, part B: per-GPU shard times of the metric's global batch, rocprof traces of
# configs 2/4/5, the LOVE rank split.
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r3prof
timeout -k 10 900 bash tools/shard_sweep.sh gpurun_out/r3prof/shards
timeout -k 10 1000 bash tools/configs_prof.sh gpurun_out/r3prof/configs_rocprof
timeout -k 10 300 python3 -u tools/love_split.py > gpurun_out/r3prof/love_split.txt 2>&1
grep -v amdgpu.ids gpurun_out/r3prof/love_split.txt
# config 5 past its start-up transient (steady-state p50 beside the driver-count mean)
timeout -k 10 600 python3 -u bench.py --model quad3d --n-train 4000 --fitc 2000 --horizon 40 --batch 512 \
    --var-inputs dynamics --steps 40 --warmup 30 --no-cpu-baseline > gpurun_out/r3prof/config5_steady.json 2>> gpurun_out/r3prof/bench_b.err
