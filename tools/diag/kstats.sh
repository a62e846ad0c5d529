# per-kernel average durations of one-stream bench steps (rocprofv3 kernel trace), for quick A/B checks
#   bash tools/diag/kstats.sh TAG [bench args...]
set -o pipefail
R=$GRAFT_REPO_ROOT
TAG=$1; shift
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/ks_$TAG -o run -- python3 $R/bench.py --no-cpu --streams 1 --iso-steps 0 --host-steps 0 --steps 20 "$@" > $R/gpurun_out/ks_$TAG.json 2> $R/gpurun_out/ks_$TAG.err || { tail -5 $R/gpurun_out/ks_$TAG.err; exit 1; }
python3 - $R/gpurun_out/ks_$TAG/run_kernel_stats.csv <<'PY'
import csv, sys
for r in list(csv.DictReader(open(sys.argv[1])))[:12]:
    print("%-34s %6s calls  avg %9.1f us" % (r["Name"].split("(")[0].replace("void ", "")[:34], r["Calls"], float(r["AverageNs"]) / 1e3))
PY
# per-launch-shape breakdown (e.g. the pyramid's levels, the quadtree's level groups): grid size -> avg
python3 - $R/gpurun_out/ks_$TAG/run_kernel_trace.csv <<'PY'
import csv, sys, collections
d = collections.defaultdict(list)
for r in csv.DictReader(open(sys.argv[1])):
    n = r["Kernel_Name"].split("(")[0].replace("void ", "")
    if "pyramid" in n or "fast" in n or "quadtree" in n or "qt_" in n:
        d[(n, int(r.get("Grid_Size_X", r.get("Grid_Size", 0))) * int(r.get("Grid_Size_Y", 1)) * int(r.get("Grid_Size_Z", 1)),
           int(r.get("LDS_Block_Size", r.get("Lds_Size", 0)) or 0))].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
for k in sorted(d):
    print("%-34s grid %8d lds %6d  %5d calls  avg %8.1f us" % (k[0][:34], k[1], k[2], len(d[k]), sum(d[k]) / len(d[k])))
PY
