set -e
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/prof_r1
# bench already captured above in the first call
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_r1/stats -o run -- python bench.py --steps 30 --warmup 20 --no-cpu-baseline > gpurun_out/prof_r1/stats.log 2>&1
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d gpurun_out/prof_r1/fetch -o run -- python bench.py --steps 10 --warmup 20 --no-cpu-baseline > gpurun_out/prof_r1/fetch.log 2>&1
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d gpurun_out/prof_r1/write -o run -- python bench.py --steps 10 --warmup 20 --no-cpu-baseline > gpurun_out/prof_r1/write.log 2>&1
ls -R gpurun_out/prof_r1 | head -30
