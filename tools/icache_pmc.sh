#!/bin/bash
# Instruction-fetch counters of the SQP kernel at the driver's command (run through gpurun):
#   bash tools/icache_pmc.sh OUTDIR [bench args...]
set -e
OUT=${1:?outdir}; shift
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p "$OUT"
timeout -s KILL 60 rocprofv3 --list-avail > "$OUT/avail.txt" 2>&1 || true
grep -i -E "ICACHE|IFETCH|INST_ANY|SQC_" "$OUT/avail.txt" | head -60 > "$OUT/avail_icache.txt" || true
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_IFETCH SQC_ICACHE_HITS SQC_ICACHE_MISSES \
    SQC_ICACHE_MISSES_DUPLICATE --kernel-trace --output-format csv -d "$OUT/ic" -o run -- \
    python3 bench.py --no-cpu-baseline "$@" > "$OUT/ic.log" 2>&1
python3 - "$OUT" <<'PY'
import csv, glob, sys, collections
f = glob.glob(sys.argv[1] + "/ic/**/*counter_collection.csv", recursive=True)
acc = collections.defaultdict(list)
for r in csv.DictReader(open(f[0])):
    if "sqp_step" in r["Kernel_Name"]:
        acc[r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, v in acc.items():
    print(k, len(v), sum(v[-20:]) / min(20, len(v)))
PY
