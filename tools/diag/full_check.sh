# Every GPU test (the node-list quadtree, then the parity tests again with the path-code kernel), FETCH of
# the default library and an alternative build, and alternating bench lines of both.
#   bash tools/diag/full_check.sh TAG DIR   (DIR under orb-slam-_amd/)
set -o pipefail
R=$GRAFT_REPO_ROOT
TAG=$1; D=$2
cd $R
timeout -k 10 600 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/fc_$TAG.log 2>&1 || { tail -30 gpurun_out/fc_$TAG.log; exit 1; }
echo "all gpu tests: $(tail -1 gpurun_out/fc_$TAG.log)"
ORBX_QT_PATHS=1 timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fuzz.py -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/fcp_$TAG.log 2>&1 || { tail -30 gpurun_out/fcp_$TAG.log; exit 1; }
echo "path-code quadtree: $(tail -1 gpurun_out/fcp_$TAG.log)"
bash tools/diag/fetch_libs.sh $TAG $D | grep -E "quadtree|fast" || exit 1
bash tools/diag/kstats_libs.sh $TAG $D | grep -E "==|fast_cells|describe|quadtree|^default|^build" || exit 1
