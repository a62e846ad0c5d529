# A/B of environment settings on the default build (isolated stage times), two rounds in alternating order:
#   bash tools/diag/env_ab.sh "" "ORBX_PYR_PAIRS=12" ...     (on the GPU box)
set -o pipefail
cd $GRAFT_REPO_ROOT
for i in 1 2; do
  for e in "$@"; do
    env $e timeout -k 10 300 python bench.py --no-cpu --host-steps 0 --ingress-peers 0 --steps 20 --warmup 5 > gpurun_out/envab.json 2>gpurun_out/envab.err || exit 1
    python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(repr(sys.argv[2]), d['value'], d['ms_per_step'], d['stage_ms_isolated'])" gpurun_out/envab.json "$e"
  done
done
