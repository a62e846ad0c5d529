# Round 5 A/B: parity subset per alternative library (ORBX_LIB), then alternating pipelined bench lines,
# then one-stream kernel stats per library.
#   bash tools/r5/ab.sh TAG DIR1 [DIR2 ...]     (DIRs under orb-slam-_amd/, from tools/diag/build_alt.sh)
set -o pipefail
R=$GRAFT_REPO_ROOT
TAG=$1; shift
O=$R/gpurun_out/r5ab_$TAG
mkdir -p $O
cd $R
for L in "$@"; do
  export ORBX_LIB=$R/orb-slam-_amd/$L/liborbx.so
  timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fuzz.py tests/test_gpu_init.py -x -q -m gpu --timeout 120 --timeout-method thread > $O/pt_$L.log 2>&1 || { echo PYTEST_FAIL $L; tail -30 $O/pt_$L.log; exit 1; }
  echo "$L: $(tail -1 $O/pt_$L.log)"
done
unset ORBX_LIB
for i in 1 2; do
  for L in default "$@"; do
    if [ $L = default ]; then unset ORBX_LIB; else export ORBX_LIB=$R/orb-slam-_amd/$L/liborbx.so; fi
    timeout -k 10 300 python bench.py --no-cpu --host-steps 0 --steps 20 --warmup 5 > $O/b_${L}_${i}.json 2> $O/b.err || { echo BENCH_FAIL; tail -20 $O/b.err; exit 1; }
    python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], d['value'], d['ms_per_step'], d['stage_ms_isolated'])" $O/b_${L}_${i}.json $L
  done
done
for L in default "$@"; do
  if [ $L = default ]; then unset ORBX_LIB; else export ORBX_LIB=$R/orb-slam-_amd/$L/liborbx.so; fi
  bash tools/diag/kstats.sh r5ab_${TAG}_$L > $O/ks_$L.txt 2>&1 || { echo KS_FAIL; tail -20 $O/ks_$L.txt; exit 1; }
  echo "== $L"; grep -E "quadtree|describe|blur|fast|pyramid" $O/ks_$L.txt | head -24
done
