#!/bin/bash
# LDS counters of the SQP kernel at the driver's command (one SQ pass): bank-conflict cycles against
# all LDS-array cycles, LDS instructions, LDS issue stalls.  bash tools/lds_pmc.sh OUTDIR
OUT=${1:?outdir}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 2
mkdir -p "$OUT"
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE \
    SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_WAIT_ANY --kernel-trace --output-format csv -d "$OUT/lds" -o run -- \
    python3 bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline > "$OUT/lds.log" 2>&1 || exit $?
python3 - "$OUT" <<'PY'
import csv, glob, sys, collections
o = sys.argv[1]
f = glob.glob(f"{o}/lds/**/run_counter_collection.csv", recursive=True)[0]
acc = collections.defaultdict(lambda: collections.defaultdict(float)); n = collections.Counter()
for r in csv.DictReader(open(f)):
    k = r["Kernel_Name"]
    if "sqp_step" not in k and "var_tri" not in k: continue
    acc[k][r["Counter_Name"]] += float(r["Counter_Value"]); n[(k, r["Counter_Name"])] += 1
for k, d in acc.items():
    c = n[(k, "SQ_WAVE_CYCLES")]
    print(k[:60], "dispatches", c)
    for name, v in sorted(d.items()): print(f"   {name:24s} {v / max(c, 1):16.0f} per dispatch")
PY
