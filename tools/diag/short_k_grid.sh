# The driver's bench invocation (--steps 20 --warmup 5) over batch sizes and stream counts, alternating.
#   bash tools/diag/short_k_grid.sh
set -o pipefail
cd $GRAFT_REPO_ROOT
for i in 1 2; do
  for cfg in "384 3" "512 3" "768 3" "384 2" "512 2" "384 4"; do
    set -- $cfg
    timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu --host-steps 0 --iso-steps 0 --batch $1 --streams $2 > gpurun_out/skg.json 2>gpurun_out/skg.err || { tail -20 gpurun_out/skg.err; exit 1; }
    python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print('K20 batch', sys.argv[2], 'streams', sys.argv[3], d['value'], d['ms_per_step'])" gpurun_out/skg.json $1 $2
  done
done
