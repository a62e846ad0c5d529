# bench.py's frames per step and pipeline depth, one short run each (no CPU leg, no isolated pass):
#   bash tools/diag/batch_stream_sweep.sh "1024 3" "2048 3" ...     (on the GPU box)
set -o pipefail
cd $GRAFT_REPO_ROOT
for cfg in "$@"; do
  set -- $cfg
  timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-cpu --ingress-peers 0 --host-steps 0 --iso-steps 0 --batch $1 --streams $2 > gpurun_out/sw_$1_$2.json 2> gpurun_out/sw_$1_$2.err || exit 1
  python3 -c "import json; d=json.load(open('gpurun_out/sw_$1_$2.json')); print('$1 $2', d['value'], d['ms_per_step'])"
done
