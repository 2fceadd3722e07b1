#!/bin/bash
# Config-5 iteration pass (run through gpurun from the repo root): bash tools/c5_check.sh OUTDIR [pytest -k expr]
# quad3d GPU parity tests, the config-5 bench line (exact variance, --steps 20 --warmup 5) and its phase table.
set -e
OUT=${1:?outdir}; K=${2:-quad3d}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p "$OUT"
[ "$K" = none ] || timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q -k "$K" --timeout 300 --timeout-method thread > "$OUT/pytest.log" 2>&1 || { tail -40 "$OUT/pytest.log"; exit 1; }
[ "$K" = none ] || tail -2 "$OUT/pytest.log"
timeout -k 10 300 python3 bench.py --model quad3d --n-train 4000 --fitc 2000 --horizon 40 --batch 512 \
    --var-inputs dynamics --steps 20 --warmup 5 --no-cpu-baseline > "$OUT/config5.json" 2> "$OUT/config5.err"
python3 -c "import json; d=json.load(open('$OUT/config5.json')); print('value', round(d['value']), 'sqp', round(d['kernel_ms_per_step']['sqp'],3), 'var', round(d['kernel_ms_per_step']['variance'],3), 'sqp it', d['sqp_iter_mean'], d['sqp_iter_max'], 'qp', d['qp_iter_mean_per_step'], d['qp_iter_max_per_step'], d['status_counts'])"
if [ -f gp-mpc_amd/gpmpc/lib/libgpmpc_mi355x_timing.so ]; then
  GPMPC_LIB=$GRAFT_REPO_ROOT/gp-mpc_amd/gpmpc/lib/libgpmpc_mi355x_timing.so timeout -k 10 300 python3 tools/phase_timing.py \
      --model quad3d --n-train 4000 --fitc 2000 --horizon 40 --batch 512 --var-inputs dynamics --warmup 3 --steps 3 > "$OUT/phase5.txt" 2>&1
  cat "$OUT/phase5.txt"
fi
