# bench.py --no-cpu at several step counts (timed-region length vs pipeline ramp effects)
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R
for k in 20 60 200; do
  timeout -k 10 200 python bench.py --no-cpu --steps $k > gpurun_out/steps_$k.json 2>gpurun_out/steps_$k.err || { tail -20 gpurun_out/steps_$k.err; exit 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/steps_$k.json')); print($k, d['value'], d['ms_per_step'])"
done
