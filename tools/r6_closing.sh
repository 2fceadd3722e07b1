#!/bin/bash
# Round-6 closing evidence on the final kernel: full GPU suite + smoke + bench (tools/r6_check.sh), then the
# driver's command profiled (tools/driver_prof.sh).  bash tools/r6_closing.sh OUTDIR
OUT=${1:?outdir}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 2
mkdir -p "$OUT"
bash tools/r6_check.sh "$OUT/check"
rc=$?
if [ $rc -ne 0 ]; then exit $rc; fi
bash tools/driver_prof.sh "$OUT/driver_cmd" > "$OUT/driver_prof.log" 2>&1 || exit $?
tail -c 400 "$OUT/driver_cmd/bench.json"
