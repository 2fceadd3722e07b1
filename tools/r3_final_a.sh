#!/bin/bash
# Round-3 evidence, part A: the GPU suite, then tools/round_profile.sh into gpurun_out/r3prof.
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r3prof
timeout -k 10 900 python3 -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > gpurun_out/r3prof/pytest_gpu.log 2>&1 || { tail -40 gpurun_out/r3prof/pytest_gpu.log; exit 1; }
tail -2 gpurun_out/r3prof/pytest_gpu.log
bash tools/round_profile.sh gpurun_out/r3prof
python3 - <<'PY'
import json
for f in ["driver/bench", "config2", "config4", "config5", "config4_exact", "config5_exact"]:
    d = json.loads([x for x in open(f"gpurun_out/r3prof/{f}.json") if x.startswith("{")][-1])
    print(f, round(d["value"]), d["kernel_ms_per_step"], d["sqp_iter_mean"], (d.get("cpu_baseline") or {}).get("value"), d["status_counts"])
PY
