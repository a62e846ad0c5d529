"""Summarise rocprofv3 FETCH_SIZE / WRITE_SIZE passes per kernel.

Units: rocprofv3 reports FETCH_SIZE / WRITE_SIZE in KiB per dispatch.  On gfx950
FETCH_SIZE tallies 64 B per 128-B memory-side read request, i.e. half the bytes of a
coalesced read (MI355X_MICROARCH.md "HBM"); our kernels read whole coalesced rows
(dword loads and LDS-DMA, 256 B per wave instruction), so reads are doubled.  Writes
are counted exactly.  Both the raw and the corrected figures are kept.

Writes <dir>/pmc_summary.json and, with --profiles OUT, the file bench.py reads for
roofline.traffic (profiles/pmc_traffic.json).
"""
import argparse
import csv
import glob
import json
import os
import sys
from collections import defaultdict

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from srchash import kernel_sources_sha256  # noqa: E402


def load(counter_dir, counter):
    files = glob.glob(os.path.join(counter_dir, "**", "*counter_collection.csv"), recursive=True)
    per = defaultdict(list)
    for fn in files:
        for r in csv.DictReader(open(fn)):
            if r.get("Counter_Name") != counter:
                continue
            name = r["Kernel_Name"].split("(")[0].split("::")[-1]
            per[name].append(float(r["Counter_Value"]))
    return per


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dir")
    ap.add_argument("--batch", type=int, default=None, help="frames per step (default: bench.py's DEFAULT_BATCH)")
    ap.add_argument("--profiles", default=None)
    a = ap.parse_args()
    if a.batch is None:
        from srchash import bench_default_batch
        a.batch = bench_default_batch()
    fetch = load(os.path.join(a.dir, "FETCH_SIZE"), "FETCH_SIZE")
    write = load(os.path.join(a.dir, "WRITE_SIZE"), "WRITE_SIZE")
    out = {}
    for k in sorted(set(fetch) | set(write)):
        f = fetch.get(k, [])
        w = write.get(k, [])
        fk = sum(f) / len(f) if f else 0.0
        wk = sum(w) / len(w) if w else 0.0
        out[k] = {"dispatches": len(f) or len(w), "fetch_kib_raw": round(fk, 1), "write_kib": round(wk, 1),
                  "bytes_per_launch_raw": int((fk + wk) * 1024),
                  "bytes_per_launch": int((2 * fk + wk) * 1024)}
    json.dump(out, open(os.path.join(a.dir, "pmc_summary.json"), "w"), indent=1)
    print(json.dumps(out, indent=1))
    if a.profiles:
        doc = {"batch": a.batch, "source": "rocprofv3 --pmc FETCH_SIZE / --pmc WRITE_SIZE (separate passes) of "
               "python3 bench.py --steps 5 --warmup 1 --no-cpu --batch %d" % a.batch,
               "bytes_per_launch": "2 x FETCH_SIZE + WRITE_SIZE (KiB x 1024), averaged over dispatches",
               "kernel_sources_sha256": kernel_sources_sha256(), "kernels": out}
        json.dump(doc, open(a.profiles, "w"), indent=1)


if __name__ == "__main__":
    main()
