# Quick per-kernel timing: rocprofv3 kernel-trace stats of a short bench run (no tests).
# usage: bash tools/gpu_prof.sh TAG [BATCH]
set -o pipefail
R=$GRAFT_REPO_ROOT
TAG=${1:-p}
B=${2:-192}
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/kt_$TAG -o run -- python3 $R/bench.py --batch $B --steps 10 --warmup 2 --no-cpu > $R/gpurun_out/kt_$TAG.json 2> $R/gpurun_out/kt_$TAG.err || { echo PROF_FAIL; tail -20 $R/gpurun_out/kt_$TAG.err; exit 1; }
python3 - $R/gpurun_out/kt_$TAG/run_kernel_stats.csv <<'EOF'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
for r in rows[:16]:
    print("%-40s %6s calls  avg %9.1f us  tot %5.1f%%" % (r["Name"].split("(")[0][:40], r["Calls"], float(r["AverageNs"]) / 1e3, float(r["Percentage"])))
EOF
