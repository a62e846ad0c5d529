# bench.py at its defaults plus extra options, one short run each (no CPU leg, no isolated pass):
#   bash tools/diag/opt_sweep.sh "" "--match-stream" ...     (on the GPU box)
set -o pipefail
cd $GRAFT_REPO_ROOT
i=0
for opts in "$@"; do
  i=$((i+1))
  timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-cpu --ingress-peers 0 --host-steps 0 --iso-steps 0 $opts > gpurun_out/os_$i.json 2> gpurun_out/os_$i.err || exit 1
  python3 -c "import json,sys; d=json.load(open('gpurun_out/os_$i.json')); print(repr(sys.argv[1]), d['value'], d['ms_per_step'])" "$opts"
done
