# config-1 host path: wall latency, then per-kernel durations and the per-call timeline under rocprofv3
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R && timeout -k 10 120 python tools/diag/host_latency.py 1000 || exit 1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d $R/gpurun_out/hl -o run -- python3 $R/tools/diag/host_latency.py 200 > $R/gpurun_out/hl.txt 2>&1 || { tail $R/gpurun_out/hl.txt; exit 1; }
python3 - $R/gpurun_out/hl <<'PY'
import csv, glob, sys, collections
d = sys.argv[1]
ev = []
for f in glob.glob(d + "/**/*kernel_trace.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        ev.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"].split("(")[0].replace("void ", "")[:40]))
for f in glob.glob(d + "/**/*memory_copy_trace.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        ev.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), "copy " + r.get("Direction", "").replace("MEMORY_COPY_", "")))
ev.sort()
# one call = from a H2D copy to the next H2D copy; report the last 5 calls' timelines and per-name averages
starts = [i for i, e in enumerate(ev) if "HOST_TO_DEVICE" in e[2] or "H2D" in e[2] or "HostToDevice" in e[2]]
print("events", len(ev), "calls", len(starts))
agg = collections.defaultdict(list)
calls = []
for a, b in zip(starts[-101:-1], starts[-100:]):
    seg = ev[a:b]
    t0 = seg[0][0]
    calls.append(seg[-1][1] - t0)
    for s, e, n in seg:
        agg[n].append(e - s)
for s, e, n in ev[starts[-2]:starts[-1]]:
    print("  +%7.1f us  %7.1f us  %s" % ((s - ev[starts[-2]][0]) / 1e3, (e - s) / 1e3, n))
print("first copy -> last op end per call: %.1f us" % (sum(calls) / len(calls) / 1e3))
for n, v in sorted(agg.items(), key=lambda x: -sum(x[1])):
    print("%-42s %5d  avg %7.1f us" % (n, len(v), sum(v) / len(v) / 1e3))
PY
