set -o pipefail
cd $GRAFT_REPO_ROOT
for cfg in "192 3" "256 3" "384 3" "192 4" "256 4" "128 4"; do
  set -- $cfg
  timeout -k 10 120 python bench.py --no-cpu --batch $1 --streams $2 --pool 3 --steps 20 > gpurun_out/sw_$1_$2.json 2> gpurun_out/sw_$1_$2.err || { echo FAIL $cfg; tail -3 gpurun_out/sw_$1_$2.err; exit 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/sw_$1_$2.json')); print('$1 $2', d['value'], d['ms_per_step'])"
done
