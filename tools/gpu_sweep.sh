# Throughput sweep over frames per step and pipeline depth (no CPU baseline).
#   bash tools/gpu_sweep.sh "192 3" "256 3" ...
set -o pipefail
cd $GRAFT_REPO_ROOT
for cfg in "$@"; do
  set -- $cfg
  timeout -k 10 120 python bench.py --no-cpu --batch $1 --streams $2 --steps 20 > gpurun_out/sw_$1_$2.json 2> gpurun_out/sw_$1_$2.err || { echo FAIL $cfg; tail -3 gpurun_out/sw_$1_$2.err; exit 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/sw_$1_$2.json')); print('$1 $2', d['value'], d['ms_per_step'])"
done
