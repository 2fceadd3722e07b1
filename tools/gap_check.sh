#!/bin/bash
# Dispatch gaps between the step's kernels (bench with events, rocprofv3 kernel trace):
#   bash tools/gap_check.sh OUTDIR
set -e
OUT=${1:?outdir}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p "$OUT"
A="--gpus 1 --steps 20 --warmup 5 --no-cpu-baseline"
for rep in 1 2; do
GPMPC_EVENT_FENCE=1 timeout -k 10 120 python3 bench.py $A > "$OUT/bench_fence_$rep.json" 2> "$OUT/bench_fence_$rep.err"
timeout -k 10 120 python3 bench.py $A > "$OUT/bench_nofence_$rep.json" 2> "$OUT/bench_nofence_$rep.err"
done
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d "$OUT/trace" -o run -- \
    python3 bench.py $A > "$OUT/trace.log" 2>&1
python3 - "$OUT" <<'PY'
import csv, glob, json, sys
o = sys.argv[1]
for f in sorted(glob.glob(o + "/bench_*.json")):
    d = json.loads([x for x in open(f) if x.startswith("{")][-1])
    print(f, round(d["value"]), d["ms_per_step"], d["kernel_ms_per_step"])
rows = [r for r in csv.DictReader(open(glob.glob(o + "/trace/*kernel_trace.csv")[0])) if "gpmpc" in r["Kernel_Name"]]
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
pe = None
for r in rows[-6:]:
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    print(r["Kernel_Name"][:36], "dur %.2f gap %.2f" % ((e - s) / 1e3, (s - pe) / 1e3 if pe else 0))
    pe = e
PY
