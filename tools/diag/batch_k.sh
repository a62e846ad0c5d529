# Bench lines at the driver's K = 20 and the default K = 100 over batch sizes (alternating).
#   bash tools/diag/batch_k.sh "768 1024 1536"
set -o pipefail
cd $GRAFT_REPO_ROOT
BS=${1:-"768 1024 1536"}
for i in 1 2; do
  for B in $BS; do
    timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu --host-steps 0 --iso-steps 0 --batch $B > gpurun_out/bk.json 2>gpurun_out/bk.err || { tail -20 gpurun_out/bk.err; exit 1; }
    python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print('K20 batch', sys.argv[2], d['value'], d['ms_per_step'])" gpurun_out/bk.json $B
  done
done
for B in $BS; do
  timeout -k 10 300 python bench.py --no-cpu --host-steps 0 --iso-steps 0 --batch $B > gpurun_out/bk.json 2>gpurun_out/bk.err || { tail -20 gpurun_out/bk.err; exit 1; }
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print('K100 batch', sys.argv[2], d['value'], d['ms_per_step'])" gpurun_out/bk.json $B
done
