# The driver's bench invocation (--steps 20 --warmup 5) at several batch sizes, alternating, to see the
# pipeline ramp at short K against the batch size.
#   bash tools/diag/short_k_sweep.sh "256 384 512"
set -o pipefail
cd $GRAFT_REPO_ROOT
BS=${1:-"256 384 512"}
for i in 1 2; do
  for B in $BS; do
    timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu --host-steps 0 --iso-steps 0 --batch $B > gpurun_out/sk.json 2>gpurun_out/sk.err || { tail -20 gpurun_out/sk.err; exit 1; }
    python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print('K20 batch', sys.argv[2], d['value'], d['ms_per_step'])" gpurun_out/sk.json $B
  done
done
