# Iteration run: GPU parity tests, a no-CPU bench line, per-kernel stats, HBM PMC passes.
#   bash tools/gpu_iter.sh TAG [pmc]
set -o pipefail
R=$GRAFT_REPO_ROOT
TAG=${1:-it}
cd $R
timeout -k 10 600 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu_$TAG.log 2>&1 || { echo PYTEST_FAIL; tail -40 gpurun_out/pytest_gpu_$TAG.log; exit 1; }
tail -1 gpurun_out/pytest_gpu_$TAG.log
timeout -k 10 300 python bench.py --no-cpu > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err || { echo BENCH_FAIL; tail -20 gpurun_out/bench_$TAG.err; exit 1; }
cat gpurun_out/bench_$TAG.json
bash tools/gpu_prof.sh $TAG || exit 1
if [ "$2" = "pmc" ]; then bash tools/collect_pmc.sh $TAG > gpurun_out/pmc_$TAG.log 2>&1 || { echo PMC_FAIL; tail -20 gpurun_out/pmc_$TAG.log; exit 1; }
  python3 -c "
import json; d=json.load(open('$R/gpurun_out/pmc_$TAG/pmc_summary.json'))
for k,v in d.items():
    if k.startswith('k_'): print('%-18s %6.1f MB/launch (raw fetch %.1f MB, write %.1f MB)' % (k, v['bytes_per_launch']/1e6, v['fetch_kib_raw']*1024/1e6, v['write_kib']*1024/1e6))"
fi
