# Iteration loop: GPU parity tests, a no-CPU bench line, and a one-stream kernel trace with the
# per-dispatch-shape averages (pyramid levels, quadtree groups) of the extract kernels.
#   bash tools/gpu_ab.sh TAG [pytest -k expr]
set -o pipefail
R=$GRAFT_REPO_ROOT
TAG=${1:-ab}
K=${2:-}
O=$R/gpurun_out/ab_$TAG
mkdir -p $O
cd $R
if [ -n "$K" ]; then
  timeout -k 10 300 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread -k "$K" > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
else
  timeout -k 10 300 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
fi
tail -1 $O/pytest.log
timeout -k 10 200 python bench.py --no-cpu > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
python3 -c "import json; d=json.load(open('$O/bench.json')); print('value', d['value'], 'ms/step', d['ms_per_step']); print('isolated', d['stage_ms_isolated'])"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 $R/bench.py --no-cpu --streams 1 --host-steps 0 --steps 20 > $O/bench_prof.json 2> $O/bench_prof.err || { echo PROF_FAIL; tail -20 $O/bench_prof.err; exit 1; }
python3 $R/tools/trace_shapes.py $O/prof/run_kernel_trace.csv
