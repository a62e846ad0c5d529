# Round 5 quick check: GPU parity suite, then one no-CPU bench line.
#   bash tools/r5/check.sh TAG
set -o pipefail
R=$GRAFT_REPO_ROOT
TAG=${1:-c}
O=$R/gpurun_out/r5_$TAG
mkdir -p $O
cd $R
timeout -k 10 400 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || { echo PYTEST_FAIL; tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
timeout -k 10 300 python bench.py --no-cpu --host-steps 0 --steps 20 --warmup 5 > $O/b.json 2> $O/b.err || { echo BENCH_FAIL; tail -20 $O/b.err; exit 1; }
python3 -c "import json; d=json.load(open('$O/b.json')); print(d['value'], d['ms_per_step'], d['stage_ms_isolated'], d['roofline'].get('hbm_copy_GBps'))"
