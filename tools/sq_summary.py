"""Per-kernel SQ counter averages from a rocprofv3 --pmc run (counter_collection.csv).
   python tools/sq_summary.py DIR"""
import csv
import glob
import os
import sys
from collections import defaultdict

d = sys.argv[1]
save = sys.argv[sys.argv.index("--save") + 1] if "--save" in sys.argv else None
vals = defaultdict(lambda: defaultdict(list))
for fn in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
    for r in csv.DictReader(open(fn)):
        k = r["Kernel_Name"].split("(")[0].split("::")[-1]
        vals[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, c in sorted(vals.items()):
    if not k.startswith("k_"):
        continue
    avg = {n: sum(v) / len(v) for n, v in c.items()}
    w = avg.get("SQ_WAVES", 0) or 1
    print("%-18s " % k + "  ".join("%s=%.4g" % (n.replace("SQ_", ""), v) for n, v in sorted(avg.items())))
    if "SQ_WAVE_CYCLES" in avg:
        wc = avg["SQ_WAVE_CYCLES"]
        print("%18s  per-wave: cycles %.0f, valu %.0f, lds %.0f, salu %.0f; wait_any %.2f, wait_inst %.2f, "
              "active_valu %.2f" % ("", wc / w, avg.get("SQ_INSTS_VALU", 0) / w, avg.get("SQ_INSTS_LDS", 0) / w,
                                    avg.get("SQ_INSTS_SALU", 0) / w, avg.get("SQ_WAIT_ANY", 0) / max(wc, 1),
                                    avg.get("SQ_WAIT_INST_ANY", 0) / max(wc, 1),
                                    avg.get("SQ_ACTIVE_INST_VALU", 0) / max(wc, 1)))

if save:
    import json
    import os
    sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
    from srchash import bench_default_batch, kernel_sources_sha256
    out = {}
    for k, c in vals.items():
        if k.startswith("k_"):
            out[k] = {n: sum(v) / len(v) for n, v in c.items()}
            out[k]["dispatches"] = len(next(iter(c.values())))
    json.dump({"batch": bench_default_batch(), "source": "rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU "
               "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU -- python3 bench.py --steps 3 "
               "--warmup 1 --no-cpu --streams 1 --iso-steps 0 (tools/gpu_sq.sh)",
               "kernel_sources_sha256": kernel_sources_sha256(), "per_dispatch_averages": out},
              open(save, "w"), indent=1)
