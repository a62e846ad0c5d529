# one-stream kernel stats of alternative libraries (no parity: diagnostic builds may be wrong on purpose)
#   bash tools/r5/kslibs.sh TAG DIR1 [DIR2 ...]
set -o pipefail
R=$GRAFT_REPO_ROOT
TAG=$1; shift
cd $R
for L in default "$@"; do
  if [ $L = default ]; then unset ORBX_LIB; else export ORBX_LIB=$R/orb-slam-_amd/$L/liborbx.so; fi
  bash tools/diag/kstats.sh r5k_${TAG}_$L > gpurun_out/r5k_${TAG}_$L.txt 2>&1 || { echo KS_FAIL $L; tail -20 gpurun_out/r5k_${TAG}_$L.txt; exit 1; }
  echo "== $L"; grep -E "^orbx::k_(describe|blur|fast_cells<40, 8> +1)" gpurun_out/r5k_${TAG}_$L.txt | head -4
done
