#!/bin/bash
# Round-6: configs 2 / 4 / 5 (and 5 sequential) on the final kernel, rocprofv3 kernel traces.
# bash tools/r6_configs_final.sh OUTDIR
set -e
OUT=${1:?outdir}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p "$OUT"
bash tools/configs_prof.sh "$OUT"
bash tools/r5_config5_seq.sh "$OUT"
for c in c2 c4 c5 c5seq; do
  python3 -c "
import json
l=[x for x in open('$OUT/$c.log') if x.startswith('{\"metric\"')][-1]; d=json.loads(l)
print('$c', round(d['value']), d.get('kernel_ms_per_step'), d['status_counts']['0'])"
done
