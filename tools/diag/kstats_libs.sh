# One-stream kernel times of the default library and alternative builds (tools/diag/build_alt.sh), then
# alternating pipelined bench lines of each.
#   bash tools/diag/kstats_libs.sh TAG DIR1 [DIR2 ...]   (DIRs under orb-slam-_amd/)
set -o pipefail
R=$GRAFT_REPO_ROOT
TAG=$1; shift
cd $R
for L in default "$@"; do
  if [ $L = default ]; then unset ORBX_LIB; else export ORBX_LIB=$R/orb-slam-_amd/$L/liborbx.so; fi
  bash tools/diag/kstats.sh ${TAG}_$L > gpurun_out/ks_${TAG}_$L.txt || exit 1
  echo "== $L"; head -9 gpurun_out/ks_${TAG}_$L.txt
done
for i in 1 2; do
  for L in default "$@"; do
    if [ $L = default ]; then unset ORBX_LIB; else export ORBX_LIB=$R/orb-slam-_amd/$L/liborbx.so; fi
    timeout -k 10 300 python bench.py --no-cpu --host-steps 0 --iso-steps 0 > gpurun_out/kl.json 2> gpurun_out/kl.err || { tail -5 gpurun_out/kl.err; exit 1; }
    python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], d['value'], d['ms_per_step'])" gpurun_out/kl.json $L
  done
done
