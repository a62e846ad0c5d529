# Full round measurement on one GPU: smoke, GPU parity tests, HBM PMC passes and SQ counters
# (written into profiles/ first, so the bench line carries them), the bench line with the
# CPU baseline, and the rocprofv3 kernel-trace summary of the same bench command.
#   bash tools/gpu_round.sh TAG   -> gpurun_out/round_TAG/
set -o pipefail
R=$GRAFT_REPO_ROOT
TAG=${1:-r}
O=$R/gpurun_out/round_$TAG
mkdir -p $O
cd $R
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo SMOKE_FAIL; tail -30 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 600 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { echo PYTEST_FAIL; tail -40 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
bash tools/collect_pmc.sh $TAG > $O/pmc.log 2>&1 || { echo PMC_FAIL; tail -20 $O/pmc.log; exit 1; }
cp $R/gpurun_out/pmc_$TAG/pmc_traffic.json $R/profiles/pmc_traffic.json && cp $R/gpurun_out/pmc_$TAG/pmc_traffic.json $O/
bash tools/gpu_sq.sh sq_$TAG > $O/sq.txt 2>&1 || { echo SQ_FAIL; tail -20 $O/sq.txt; exit 1; }
cp $R/gpurun_out/sq_$TAG/sq_counters.json $R/profiles/sq_counters.json && cp $R/gpurun_out/sq_$TAG/sq_counters.json $O/
cd $R
timeout -k 10 600 python bench.py > $O/bench.json 2> $O/bench.err || { echo BENCH_FAIL; tail -30 $O/bench.err; exit 1; }
cat $O/bench.json
cd /tmp && export TMPDIR=/tmp
# one stream: kernel durations are the kernels' own (bench.py's roofline timing)
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 $R/bench.py --no-cpu --streams 1 --host-steps 0 > $O/bench_prof.json 2> $O/bench_prof.err || { echo PROF_FAIL; tail -20 $O/bench_prof.err; exit 1; }
# the pipelined default command as well (durations stretched by the concurrent streams)
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_pipelined -o run -- python3 $R/bench.py --no-cpu --host-steps 0 > $O/bench_prof_pipelined.json 2> $O/bench_prof_pipelined.err || { echo PROF_FAIL; tail -20 $O/bench_prof_pipelined.err; exit 1; }
python3 - $O/prof/run_kernel_stats.csv <<'PY'
import csv, sys
for r in list(csv.DictReader(open(sys.argv[1])))[:14]:
    print("%-34s %6s calls  avg %9.1f us  tot %5.1f%%" % (r["Name"].split("(")[0][:34], r["Calls"], float(r["AverageNs"]) / 1e3, float(r["Percentage"])))
PY
