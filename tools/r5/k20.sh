# The driver's bench form (K = 20, W = 5) twice, then the secondary configs (1, 3, 5) on one GPU.
#   bash tools/r5/k20.sh TAG   -> gpurun_out/r5k20_TAG/
set -o pipefail
R=$GRAFT_REPO_ROOT
TAG=${1:-k}
O=$R/gpurun_out/r5k20_$TAG
mkdir -p $O
cd $R
for i in 1 2; do
  timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $O/bench_k20_$i.json 2> $O/bench_k20_$i.err || { echo BENCH_FAIL; tail -20 $O/bench_k20_$i.err; exit 1; }
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print('k20', d['value'], d['ms_per_step'])" $O/bench_k20_$i.json
done
bash tools/gpu_configs.sh r5_$TAG || exit 1
cp gpurun_out/configs_r5_$TAG.jsonl $O/
