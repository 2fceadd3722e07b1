#!/bin/bash
# (round 6: the cache is switched off through bench.py --lin-cache 0; the library reads no environment)
# Where the SQP kernel's HBM write traffic comes from (round 3): WRITE_SIZE / FETCH_SIZE passes of
# the driver's command with the linearisation cache off (GPMPC_LIN_CACHE=0), beside the committed
# passes with it on (profiles/r3/driver_cmd/pmc_summary.json).
set -e
OUT=gpurun_out/wbd
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p $OUT
ARGS="--gpus 1 --steps 20 --warmup 5 --no-cpu-baseline --lin-cache 0"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run -- python3 bench.py $ARGS > $OUT/trace.log 2>&1
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d $OUT/fetch -o run -- python3 bench.py $ARGS > $OUT/fetch.log 2>&1
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d $OUT/write -o run -- python3 bench.py $ARGS > $OUT/write.log 2>&1
python3 tools/pmc_summary.py --trace $OUT/trace --fetch $OUT/fetch --write $OUT/write --last 20 \
    --config '{"workload": "quad2d GP-MPC N=200 H=30, 1024 instances per GPU, closed loop, GPMPC_LIN_CACHE=0"}' -o $OUT/pmc_summary_nocache.json
