# Alternating pipelined bench lines only (no parity run), per alternative library: timing-only diagnostic builds
#   bash tools/r5/ab_bench.sh TAG LIB1 [LIB2 ...]
set -o pipefail
R=$GRAFT_REPO_ROOT
TAG=$1; shift
O=$R/gpurun_out/r5abb_$TAG
mkdir -p $O
cd $R
for i in 1 2 3; do
  for L in default "$@"; do
    if [ $L = default ]; then unset ORBX_LIB; else export ORBX_LIB=$R/orb-slam-_amd/$L/liborbx.so; fi
    timeout -k 10 300 python bench.py --no-cpu --host-steps 0 --steps 20 --warmup 5 > $O/b_${L}_${i}.json 2> $O/b.err || { echo BENCH_FAIL; tail -20 $O/b.err; exit 1; }
    python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], d['value'], d['ms_per_step'], d['stage_ms_per_step'])" $O/b_${L}_${i}.json $L
  done
done
