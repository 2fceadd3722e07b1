set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
bash tools/gpu_check.sh gpurun_out/r3b --gpus 1 --steps 20 --warmup 5
timeout -k 10 600 python3 -u bench.py --model quad3d --n-train 4000 --fitc 2000 --horizon 40 --batch 512 --var-inputs dynamics --steps 20 --warmup 5 > gpurun_out/r3b/config5.json 2> gpurun_out/r3b/config5.err
bash tools/shard_sweep.sh gpurun_out/r3b/shards
