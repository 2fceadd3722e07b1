#!/usr/bin/env python3
"""Summarise rocprofv3 kernel-trace / PMC CSVs of a bench.py run into per-kernel numbers.

    python tools/pmc_summary.py --trace DIR_STATS --fetch DIR_FETCH --write DIR_WRITE \
        --last K --config '{"model": "quad2d", ...}' -o profiles/rNN/pmc_summary.json

* durations: mean kernel time over the LAST K dispatches of each kernel (the bench's timed
  region; the warm-up dispatches come first), from the --kernel-trace CSV;
* traffic: FETCH_SIZE / WRITE_SIZE (kB) per dispatch over the same last-K window, each from its
  own --pmc pass.  MI355X_MICROARCH.md (HBM [CDNA4]): on gfx950 FETCH_SIZE reports 1/2 of the
  bytes of wide coalesced reads (128-B requests tallied at 64 B), WRITE_SIZE is exact for
  16-B/lane stores; both count Infinity-Cache (MALL) hits.  The summary keeps the raw values and
  a corrected HBM-side estimate = 2 x FETCH + WRITE.
"""

from __future__ import annotations

import argparse
import csv
import glob
import json
import os
from collections import defaultdict


def _rows(d: str, suffix: str):
    files = sorted(glob.glob(os.path.join(d, "**", f"*{suffix}"), recursive=True))
    for f in files:
        with open(f, newline="") as fh:
            yield from csv.DictReader(fh)


def _short(name: str) -> str:
    name = name.replace("void ", "")
    return name.split("(")[0]


def durations(d: str, last: int):
    per = defaultdict(list)
    for r in _rows(d, "kernel_trace.csv"):
        per[_short(r["Kernel_Name"])].append((int(r["Start_Timestamp"]), int(r["End_Timestamp"])))
    out = {}
    for k, v in per.items():
        v.sort()
        tail = v[-last:] if last > 0 else v
        ds = [(e - s) * 1e-3 for s, e in tail]
        out[k] = {"dispatches": len(v), "window": len(tail), "mean_us": sum(ds) / len(ds),
                  "min_us": min(ds), "max_us": max(ds)}
    return out


def counter(d: str, name: str, last: int):
    per = defaultdict(list)
    for r in _rows(d, "counter_collection.csv"):
        if r["Counter_Name"] == name:
            per[_short(r["Kernel_Name"])].append((int(r["Dispatch_Id"]), float(r["Counter_Value"])))
    out = {}
    for k, v in per.items():
        v.sort()
        tail = v[-last:] if last > 0 else v
        out[k] = {"dispatches": len(v), "window": len(tail), "mean_kB": sum(x for _, x in tail) / len(tail)}
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--trace", required=True)
    ap.add_argument("--fetch")
    ap.add_argument("--write")
    ap.add_argument("--last", type=int, default=0)
    ap.add_argument("--config", default="{}")
    ap.add_argument("-o", "--out", required=True)
    a = ap.parse_args()
    dur = durations(a.trace, a.last)
    fetch = counter(a.fetch, "FETCH_SIZE", a.last) if a.fetch else {}
    write = counter(a.write, "WRITE_SIZE", a.last) if a.write else {}
    kernels = {}
    for k in sorted(set(dur) | set(fetch) | set(write)):
        e = {"duration": dur.get(k)}
        if k in fetch:
            e["FETCH_SIZE_kB"] = fetch[k]["mean_kB"]
        if k in write:
            e["WRITE_SIZE_kB"] = write[k]["mean_kB"]
        if k in fetch and k in write:
            e["hbm_bytes_est"] = (2.0 * fetch[k]["mean_kB"] + write[k]["mean_kB"]) * 1024.0
        kernels[k] = e
    out = {"config": json.loads(a.config), "last_dispatches": a.last, "kernels": kernels,
           "note": "hbm_bytes_est = 2 x FETCH_SIZE + WRITE_SIZE (gfx950 FETCH_SIZE halving, MI355X_MICROARCH.md)"}
    os.makedirs(os.path.dirname(os.path.abspath(a.out)), exist_ok=True)
    with open(a.out, "w") as fh:
        json.dump(out, fh, indent=1)
    for k, e in kernels.items():
        d = e["duration"]
        print(f"{k[:60]:60s} {d['mean_us'] if d else float('nan'):10.2f} us  "
              f"fetch {e.get('FETCH_SIZE_kB', float('nan')):12.1f} kB  write {e.get('WRITE_SIZE_kB', float('nan')):12.1f} kB")


if __name__ == "__main__":
    main()
