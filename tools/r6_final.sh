#!/bin/bash
# Round-6 end-of-round evidence, part 1 (run through gpurun from the repo root): the driver's command
# profiled (bench line, rocprofv3 kernel trace + stats, SQ pass, FETCH / WRITE passes) and the secondary
# configs' rocprofv3 traces, config 5 also sequential.  bash tools/r6_final.sh OUTDIR
set -e
OUT=${1:?outdir}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p "$OUT"
bash tools/driver_prof.sh "$OUT/driver_cmd"
bash tools/configs_prof.sh "$OUT/configs_rocprof"
bash tools/r5_config5_seq.sh "$OUT/configs_rocprof"
echo done
