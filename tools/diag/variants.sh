# Parity (parity + fuzz GPU tests) of the default library and each alternative build, then one-stream kernel
# times and alternating pipelined bench lines of all of them (tools/diag/kstats_libs.sh).
#   bash tools/diag/variants.sh TAG DIR1 [DIR2 ...]   (DIRs under orb-slam-_amd/, from tools/diag/build_alt.sh)
set -o pipefail
R=$GRAFT_REPO_ROOT
TAG=$1; shift
cd $R
for L in default "$@"; do
  if [ $L = default ]; then unset ORBX_LIB; else export ORBX_LIB=$R/orb-slam-_amd/$L/liborbx.so; fi
  timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fuzz.py -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/pt_${TAG}_$L.log 2>&1 || { tail -20 gpurun_out/pt_${TAG}_$L.log; exit 1; }
  echo "$L $(tail -1 gpurun_out/pt_${TAG}_$L.log)"
done
unset ORBX_LIB
bash tools/diag/kstats_libs.sh $TAG "$@"
