set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/dump1
timeout -k 10 200 python3 -u -m pytest tests/test_gpu_semantics.py -x -v --timeout 120 --timeout-method thread > gpurun_out/dump1/pytest_sem.log 2>&1
timeout -k 10 120 python3 tools/phase_timing.py --warmup 5 --steps 20 --dump gpurun_out/dump1/phases.npy > gpurun_out/dump1/phase.txt 2>&1
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d gpurun_out/dump1/write -o run -- python3 bench.py --no-cpu-baseline > gpurun_out/dump1/write.log 2>&1
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d gpurun_out/dump1/fetch -o run -- python3 bench.py --no-cpu-baseline > gpurun_out/dump1/fetch.log 2>&1
