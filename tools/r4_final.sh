#!/bin/bash
# Round-4 evidence: the GPU suite, tools/round_profile.sh (driver command + rocprofv3 trace/stats,
# SQ and FETCH/WRITE passes, phase timing, configs 2/4/5) and the strong-scaling shard sweep, into
# OUTDIR (run through gpurun from the repo root): bash tools/r4_final.sh OUTDIR
set -e
OUT=${1:?outdir}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p "$OUT"
timeout -k 10 1000 python3 -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > "$OUT/pytest_gpu.log" 2>&1 || { tail -40 "$OUT/pytest_gpu.log"; exit 1; }
tail -2 "$OUT/pytest_gpu.log"
timeout -k 10 180 python3 -u -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1
bash tools/round_profile.sh "$OUT"
timeout -k 10 120 python3 tools/phase_timing.py --warmup 5 --batch 128 > "$OUT/phase_timing_b128.txt" 2>&1
bash tools/shard_sweep.sh "$OUT/shards" > "$OUT/shards.txt"
cat "$OUT/shards.txt"
python3 - "$OUT" <<'PY'
import json, sys
o = sys.argv[1]
for f in ["driver/bench", "config2", "config4", "config5", "config4_exact", "config5_exact"]:
    d = json.loads([x for x in open(f"{o}/{f}.json") if x.startswith("{")][-1])
    print(f, round(d["value"]), d["kernel_ms_per_step"], d["sqp_iter_mean"], (d.get("cpu_baseline") or {}).get("value"), d["status_counts"])
PY
