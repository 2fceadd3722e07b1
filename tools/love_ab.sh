#!/bin/bash
# LOVE variance kernel check (run through gpurun from the repo root): bash tools/love_ab.sh OUTDIR
# LOVE-root GPU parity tests, then configs 4 and 5 (default fast_pred_var variance) with the
# dedicated gp_love_kernel (default library) and with gp_post_kernel (-DGPMPC_LOVE_POST variant).
set -e
OUT=${1:?outdir}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p "$OUT"
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_parity.py -x -q -k "True" --timeout 200 --timeout-method thread \
    > "$OUT/pytest.log" 2>&1 || { tail -30 "$OUT/pytest.log"; exit 1; }
tail -2 "$OUT/pytest.log"
LIB=$GRAFT_REPO_ROOT/gp-mpc_amd/gpmpc/lib
for v in default lovepost; do
  L=$LIB/libgpmpc_mi355x.so; [ $v = lovepost ] && L=$LIB/libgpmpc_mi355x_lovepost.so
  [ -f "$L" ] || continue
  GPMPC_LIB=$L timeout -k 10 300 python3 bench.py --n-train 1000 --steps 20 --warmup 5 --no-cpu-baseline \
      > "$OUT/c4_$v.json" 2> "$OUT/c4_$v.err"
  GPMPC_LIB=$L timeout -k 10 300 python3 bench.py --model quad3d --n-train 4000 --fitc 2000 --horizon 40 --batch 512 \
      --var-inputs dynamics --steps 20 --warmup 5 --no-cpu-baseline > "$OUT/c5_$v.json" 2> "$OUT/c5_$v.err"
  for c in c4 c5; do
    python3 -c "import json; d=json.load(open('$OUT/${c}_$v.json')); print('$c $v', round(d['value']), d['kernel_ms_per_step'], d['status_counts'])"
  done
done
