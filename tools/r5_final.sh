#!/bin/bash
# Round-5 end-of-round evidence (run through gpurun from the repo root): the GPU suite, smoke(),
# the all-rank shard sweep and the secondary configs' rocprofv3 traces.  bash tools/r5_final.sh OUTDIR
set -e
OUT=${1:?outdir}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p "$OUT"
timeout -k 10 1200 python3 -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > "$OUT/pytest_gpu.log" 2>&1
timeout -k 10 300 python3 -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > "$OUT/smoke.log" 2>&1
bash tools/shard_sweep.sh "$OUT/shards_all" > "$OUT/shards_all_summary.txt" 2>&1
bash tools/configs_prof.sh "$OUT/configs_rocprof"
bash tools/r5_config5_seq.sh "$OUT/configs_rocprof"
