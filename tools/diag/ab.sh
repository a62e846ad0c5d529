# quick A/B of the current tree: extraction parity tests, one-stream kernel averages, two pipelined bench lines
#   bash tools/diag/ab.sh TAG
set -o pipefail
R=$GRAFT_REPO_ROOT
TAG=${1:-ab}
cd $R
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_init.py -x -q --timeout 120 --timeout-method thread > gpurun_out/ab_$TAG.log 2>&1 || { tail -30 gpurun_out/ab_$TAG.log; exit 1; }
tail -1 gpurun_out/ab_$TAG.log
bash tools/diag/kstats.sh $TAG > gpurun_out/ab_${TAG}_ks.txt || exit 1; head -12 gpurun_out/ab_${TAG}_ks.txt
cd $R
for i in 1 2; do
  timeout -k 10 300 python bench.py --no-cpu --host-steps 0 --iso-steps 0 > gpurun_out/ab_${TAG}_$i.json || exit 1
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print('bench', d['value'], d['ms_per_step'])" gpurun_out/ab_${TAG}_$i.json
done
