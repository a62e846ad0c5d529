"""Per-dispatch-shape average durations from a rocprofv3 kernel trace (run_kernel_trace.csv):
one line per (kernel, grid) so that e.g. the seven pyramid launches show up level by level."""
import collections
import csv
import sys


def main(path):
    rows = list(csv.DictReader(open(path)))
    d = collections.defaultdict(list)
    for r in rows:
        name = r["Kernel_Name"].split("(")[0]
        if "orbx" not in name:
            continue
        key = (name.replace("void ", "")[:40], r["Grid_Size_X"], r["Grid_Size_Y"], r["Grid_Size_Z"])
        d[key].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
    tot = collections.defaultdict(float)
    for (name, gx, gy, gz), v in sorted(d.items()):
        avg = sum(v) / len(v)
        tot[name] += avg
        print("%-40s grid %6s %6s %6s  %5d calls  avg %8.1f us" % (name, gx, gy, gz, len(v), avg))
    print("per-kernel sums of the shape averages (one step's launches):")
    for name, t in sorted(tot.items(), key=lambda kv: -kv[1]):
        print("  %-40s %8.1f us" % (name, t))


if __name__ == "__main__":
    main(sys.argv[1])
