#!/bin/bash
# SQ counters of the variance kernels at config 4 (run through gpurun from the repo root)
set -e
OUT=${1:?outdir}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p "$OUT"
timeout -k 10 300 python3 bench.py --n-train 1000 --steps 5 --warmup 2 --no-cpu-baseline > "$OUT/c4.json" 2>/dev/null
python3 -c "import json; d=json.load(open('$OUT/c4.json')); print('c4', round(d['value']), d['kernel_ms_per_step'])"
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_ACTIVE_INST_VMEM \
    --kernel-trace --output-format csv -d "$OUT/sq" -o run -- python3 bench.py --n-train 1000 --steps 3 --warmup 1 --no-cpu-baseline > "$OUT/sq.log" 2>&1
python3 - "$OUT" <<'PY'
import csv, sys, glob, collections
out = sys.argv[1]
f = glob.glob(f"{out}/sq/**/run_counter_collection.csv", recursive=True) + glob.glob(f"{out}/sq/run_counter_collection.csv")
rows = list(csv.DictReader(open(f[0])))
agg = collections.defaultdict(lambda: collections.defaultdict(float))
cnt = collections.Counter()
for r in rows:
    k = r.get("Kernel_Name", r.get("Kernel-Name", ""))
    if "love" not in k and "var_tri" not in k and "gp_post" not in k:
        continue
    agg[k][r["Counter_Name"]] += float(r["Counter_Value"])
    cnt[k] += 1
for k, v in agg.items():
    print(k[:60], {c: round(x) for c, x in v.items()})
PY
