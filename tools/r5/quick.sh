# Round 5 iteration: extraction parity, one-stream kernel stats, two pipelined bench lines.
#   bash tools/r5/quick.sh TAG [pytest -k expr]
set -o pipefail
R=$GRAFT_REPO_ROOT
TAG=${1:-q}
K=${2:-}
O=$R/gpurun_out/r5q_$TAG
mkdir -p $O
cd $R
if [ -n "$K" ]; then
  timeout -k 10 400 python -u -m pytest tests -x -q -m gpu -k "$K" --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || { echo PYTEST_FAIL; tail -40 $O/pytest.log; exit 1; }
else
  timeout -k 10 400 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || { echo PYTEST_FAIL; tail -40 $O/pytest.log; exit 1; }
fi
tail -1 $O/pytest.log
bash tools/diag/kstats.sh r5q_$TAG > $O/ks.txt 2>&1 || { echo KS_FAIL; tail -20 $O/ks.txt; exit 1; }
head -12 $O/ks.txt
for i in 1 2; do
  timeout -k 10 300 python bench.py --no-cpu --host-steps 0 --steps 20 --warmup 5 > $O/b_$i.json 2> $O/b.err || { echo BENCH_FAIL; tail -20 $O/b.err; exit 1; }
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print('bench', d['value'], d['ms_per_step'], d['stage_ms_isolated'], d['roofline'].get('hbm_copy_GBps'))" $O/b_$i.json
done
