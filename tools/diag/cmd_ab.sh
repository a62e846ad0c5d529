# parity tests of the current tree, then one-stream kernel averages of it against alternative builds
#   bash tools/diag/cmd_ab.sh PATTERN DIR...
set -o pipefail
cd $GRAFT_REPO_ROOT
K=$1; shift
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fuzz.py tests/test_gpu_init.py -x -q --timeout 120 --timeout-method thread > gpurun_out/pt_ab.log 2>&1 || { tail -30 gpurun_out/pt_ab.log; exit 1; }
tail -1 gpurun_out/pt_ab.log
bash tools/diag/kstats_alts.sh "$K" "$@"
