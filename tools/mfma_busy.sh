#!/bin/bash
# MFMA pipe utilisation of the variance and SQP kernels (round 3): one SQ pass per config with
# SQ_VALU_MFMA_BUSY_CYCLES (cycles the matrix pipe is busy, summed over SIMDs) beside GRBM_GUI_ACTIVE
# (GPU busy clocks) and the kernel durations of the same run.
set -e
OUT=${1:-gpurun_out/mfmabusy}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p $OUT
A="--steps 3 --warmup 2 --no-cpu-baseline"
C4="--n-train 1000"
C5="--model quad3d --n-train 4000 --fitc 2000 --horizon 40 --batch 512 --var-inputs dynamics"
for c in 3 4 5; do
  eval ARGS=\$C$c
  [ $c = 3 ] && ARGS=""
  timeout -s KILL 180 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_VALU GRBM_GUI_ACTIVE \
      --kernel-trace --output-format csv -d $OUT/c$c -o run -- python3 bench.py $ARGS $A > $OUT/c$c.log 2>&1
done
python3 - "$OUT" <<'PY'
import csv, glob, sys, collections
out = sys.argv[1]
for c in (3, 4, 5):
    f = glob.glob(f"{out}/c{c}/**/run_counter_collection.csv", recursive=True) + glob.glob(f"{out}/c{c}/run_counter_collection.csv")
    rows = list(csv.DictReader(open(f[0])))
    agg = collections.defaultdict(lambda: collections.defaultdict(list))
    dur = collections.defaultdict(list)
    for r in rows:
        k = r["Kernel_Name"]
        if "gpmpc" not in k:
            continue
        k = k.split("(")[0].replace("void ", "")
        agg[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
        dur[k].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-9)
    for k, v in agg.items():
        m = {n: sum(x) / len(x) for n, x in v.items()}
        d = sum(dur[k]) / len(dur[k])
        xcd_clk = m["GRBM_GUI_ACTIVE"] / 8                 # GRBM_GUI_ACTIVE sums the 8 XCDs' clocks
        simd_cycles = xcd_clk * 1024                       # busy clocks x SIMDs
        clk = xcd_clk / d / 1e9 if d > 0 else 0
        print(f"config {c} {k[:40]:40s} dur {d*1e3:.3f} ms  clk {clk:.2f} GHz  MFMA busy {m['SQ_VALU_MFMA_BUSY_CYCLES']/simd_cycles*100:.1f} % of SIMD-cycles  VALU instr/wave-cycle {m['SQ_INSTS_VALU']/max(m['SQ_WAVE_CYCLES'],1):.3f}")
PY
