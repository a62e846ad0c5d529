# K = 20 bench lines at the default batch with 3 and 2 pipeline streams, alternating.
#   bash tools/diag/stream_k.sh
set -o pipefail
cd $GRAFT_REPO_ROOT
for i in 1 2; do
  for st in 3 2; do
    timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-cpu --host-steps 0 --iso-steps 0 --streams $st > gpurun_out/sk.json 2>gpurun_out/sk.err || { tail -5 gpurun_out/sk.err; exit 1; }
    python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print('K20 streams', sys.argv[2], d['value'])" gpurun_out/sk.json $st
  done
done
