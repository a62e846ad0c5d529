# Secondary configs (1, 3, 5) on one GPU -> gpurun_out/configs_TAG.jsonl
set -o pipefail
R=$GRAFT_REPO_ROOT
TAG=${1:-c}
cd $R
: > gpurun_out/configs_$TAG.jsonl
for C in 1 3 5; do
  timeout -k 10 300 python tools/bench_configs.py --config $C >> gpurun_out/configs_$TAG.jsonl 2> gpurun_out/configs_${TAG}_$C.err || { echo CONFIG_FAIL $C; tail -20 gpurun_out/configs_${TAG}_$C.err; exit 1; }
  tail -1 gpurun_out/configs_$TAG.jsonl
done
