# one-stream kernel stats per alternative library (no parity run: timing-only diagnostic builds)
#   bash tools/r5/kslibs_only.sh TAG LIB1 [LIB2 ...]
set -o pipefail
R=$GRAFT_REPO_ROOT
TAG=$1; shift
cd $R
for L in default "$@"; do
  if [ $L = default ]; then unset ORBX_LIB; else export ORBX_LIB=$R/orb-slam-_amd/$L/liborbx.so; fi
  bash tools/diag/kstats.sh r5ko_${TAG}_$L > gpurun_out/r5ko_${TAG}_$L.txt 2>&1 || { echo KS_FAIL; tail -20 gpurun_out/r5ko_${TAG}_$L.txt; exit 1; }
  echo "== $L"; grep -E "quadtree|describe|fast|pyramid" gpurun_out/r5ko_${TAG}_$L.txt | grep -v grid | head -8
done
