"""Summarise rocprofv3 FETCH_SIZE / WRITE_SIZE passes per kernel.

Units: rocprofv3 reports FETCH_SIZE / WRITE_SIZE in KiB per dispatch.  On gfx950
FETCH_SIZE counts 64 B per 128-B request for wide (16 B/lane) streaming reads, i.e.
reads exactly half of those bytes (MI355X_MICROARCH.md "HBM"); our kernels read
with byte and dword loads, for which the counter is uncalibrated, so both the raw
and the x2-corrected read figures are reported.  Writes are counted exactly.
Writes profiles-ready JSON next to the CSVs and prints it.
"""
import csv
import glob
import json
import os
import sys
from collections import defaultdict


def load(counter_dir, counter):
    files = glob.glob(os.path.join(counter_dir, "**", "*counter_collection.csv"), recursive=True)
    per = defaultdict(list)
    for fn in files:
        for r in csv.DictReader(open(fn)):
            if r.get("Counter_Name") != counter:
                continue
            name = r["Kernel_Name"].split("(")[0]
            per[name].append(float(r["Counter_Value"]))
    return per


def main(d):
    fetch = load(os.path.join(d, "FETCH_SIZE"), "FETCH_SIZE")
    write = load(os.path.join(d, "WRITE_SIZE"), "WRITE_SIZE")
    out = {}
    for k in sorted(set(fetch) | set(write)):
        f = fetch.get(k, [])
        w = write.get(k, [])
        fk = sum(f) / len(f) if f else 0.0
        wk = sum(w) / len(w) if w else 0.0
        out[k] = {"dispatches": len(f) or len(w), "fetch_kib_raw": round(fk, 1), "write_kib": round(wk, 1),
                  "bytes_per_launch_raw": int((fk + wk) * 1024),
                  "bytes_per_launch_fetch_x2": int((2 * fk + wk) * 1024)}
    json.dump(out, open(os.path.join(d, "pmc_summary.json"), "w"), indent=1)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main(sys.argv[1])
