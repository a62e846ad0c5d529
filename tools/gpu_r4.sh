# Round-4 iteration: extraction parity first (fail fast), the whole GPU suite, then per-kernel times of the
# path-code quadtree against the node-list kernel (ORBX_QT_NODES=1) and two pipelined bench lines each.
#   bash tools/gpu_r4.sh TAG
set -o pipefail
R=$GRAFT_REPO_ROOT
TAG=${1:-r4}
cd $R
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fuzz.py tests/test_golden.py -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/pt1_$TAG.log 2>&1 || { tail -40 gpurun_out/pt1_$TAG.log; exit 1; }
tail -1 gpurun_out/pt1_$TAG.log
timeout -k 10 400 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/pt_$TAG.log 2>&1 || { tail -40 gpurun_out/pt_$TAG.log; exit 1; }
tail -1 gpurun_out/pt_$TAG.log
bash tools/diag/kstats.sh ${TAG}_paths > gpurun_out/ks_${TAG}_paths.txt || exit 1
grep -E "qt_|quadtree|fast|describe" gpurun_out/ks_${TAG}_paths.txt
ORBX_QT_NODES=1 bash tools/diag/kstats.sh ${TAG}_nodes > gpurun_out/ks_${TAG}_nodes.txt || exit 1
grep -E "qt_|quadtree" gpurun_out/ks_${TAG}_nodes.txt
for i in 1 2; do
  for M in paths nodes; do
    if [ $M = nodes ]; then export ORBX_QT_NODES=1; else unset ORBX_QT_NODES; fi
    timeout -k 10 300 python bench.py --no-cpu --host-steps 0 --iso-steps 0 > gpurun_out/b_${TAG}_$M.json 2>gpurun_out/b_${TAG}_$M.err || { tail -5 gpurun_out/b_${TAG}_$M.err; exit 1; }
    python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], d['value'], d['ms_per_step'])" gpurun_out/b_${TAG}_$M.json $M
  done
done
