#!/bin/bash
# LDS bank-conflict cycles of each Newton-system recursion in isolation (tools/ric_micro: one kernel
# per recursion and model).  bash tools/ric_lds_pmc.sh OUTDIR
OUT=${1:?outdir}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 2
mkdir -p "$OUT"
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAVE_CYCLES --kernel-trace \
    --output-format csv -d "$OUT/pmc" -o run -- ./tools/ric_micro > "$OUT/ric_micro.txt" 2>&1 || exit $?
python3 - "$OUT" <<'PY'
import csv, glob, sys, collections
o = sys.argv[1]
f = glob.glob(f"{o}/pmc/**/run_counter_collection.csv", recursive=True)[0]
acc = collections.defaultdict(lambda: collections.defaultdict(float))
for r in csv.DictReader(open(f)):
    acc[r["Kernel_Name"]][r["Counter_Name"]] += float(r["Counter_Value"])
for k, d in acc.items():
    print(k[:70], " ".join(f"{n}={v:.0f}" for n, v in sorted(d.items())),
          f"conflict/idx={d['SQ_LDS_BANK_CONFLICT'] / max(d['SQ_LDS_IDX_ACTIVE'], 1):.2f}")
PY
