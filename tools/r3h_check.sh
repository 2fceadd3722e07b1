#!/bin/bash
# Config 5 A/B (current SQP kernel vs the round-2 kernel source built against the same C-ABI),
# config-3 shard sweep (strong-scaling shards) and the LOVE rank split.
set -e
OUT=gpurun_out/r3h
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p $OUT
C5="--model quad3d --n-train 4000 --fitc 2000 --horizon 40 --batch 512 --var-inputs dynamics --steps 10 --warmup 3 --no-cpu-baseline"
timeout -k 10 400 python3 -u bench.py $C5 > $OUT/c5_cur.json 2> $OUT/c5.err
GPMPC_LIB=$PWD/gp-mpc_amd/gpmpc/lib/libgpmpc_mi355x_r2k.so timeout -k 10 400 python3 -u bench.py $C5 > $OUT/c5_r2k.json 2>> $OUT/c5.err
python3 - <<'PY'
import json
for f in ["c5_cur", "c5_r2k"]:
    d = json.loads([x for x in open(f"gpurun_out/r3h/{f}.json") if x.startswith("{")][-1])
    print(f, round(d["value"]), d["kernel_ms_per_step"], d["sqp_iter_mean"], d["qp_iter_mean_per_step"])
PY
timeout -k 10 900 bash tools/shard_sweep.sh $OUT/shards
timeout -k 10 300 python3 -u tools/love_split.py > $OUT/love_split.txt 2>&1
grep -v amdgpu.ids $OUT/love_split.txt
