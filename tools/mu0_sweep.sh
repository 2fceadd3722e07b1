set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/mu0
for m in 1.0 0.1 0.01 10.0 100.0; do
  timeout -k 10 120 python3 bench.py --no-cpu-baseline --qp-mu0 $m > gpurun_out/mu0/b_$m.json 2>/dev/null
done
python3 - <<'PY'
import json,glob
for f in sorted(glob.glob('gpurun_out/mu0/b_*.json')):
    d=json.loads([x for x in open(f) if x.startswith('{')][-1])
    print(f, round(d['value']), d['kernel_ms_per_step'], d['sqp_iter_mean'], d['qp_iter_mean_per_step'], d['status_counts'])
PY
