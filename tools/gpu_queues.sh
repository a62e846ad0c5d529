# pipeline depth vs hardware queues at the 200-step default
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R
for cfg in "4 3" "8 3" "8 4" "8 6"; do
  set -- $cfg
  GPU_MAX_HW_QUEUES=$1 timeout -k 10 200 python bench.py --no-cpu --streams $2 > gpurun_out/q_$1_$2.json 2>gpurun_out/q_$1_$2.err || { tail -20 gpurun_out/q_$1_$2.err; exit 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/q_$1_$2.json')); print('queues $1 streams $2', d['value'], d['ms_per_step'])"
done
