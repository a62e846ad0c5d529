# Quadtree iteration: extraction parity first (fail fast), per-kernel times (path-code vs node-list kernel),
# the path kernel's phase profile, and one pipelined bench line.
#   bash tools/gpu_r4q.sh TAG
set -o pipefail
R=$GRAFT_REPO_ROOT
TAG=${1:-q}
cd $R
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fuzz.py tests/test_golden.py tests/test_gpu_init.py -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/pt1_$TAG.log 2>&1 || { tail -40 gpurun_out/pt1_$TAG.log; exit 1; }
tail -1 gpurun_out/pt1_$TAG.log
bash tools/diag/kstats.sh ${TAG} > gpurun_out/ks_${TAG}.txt || exit 1
grep -E "qt_|quadtree|fast_cells<40, 10>   |describe" gpurun_out/ks_${TAG}.txt | head -20
timeout -k 10 120 python tools/diag/qp_prof.py > gpurun_out/qp_${TAG}.txt 2>&1 || { tail -5 gpurun_out/qp_${TAG}.txt; exit 1; }
cat gpurun_out/qp_${TAG}.txt
timeout -k 10 300 python bench.py --no-cpu --host-steps 0 --iso-steps 0 > gpurun_out/b_${TAG}.json 2>gpurun_out/b_${TAG}.err || { tail -5 gpurun_out/b_${TAG}.err; exit 1; }
python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print('bench', d['value'], d['ms_per_step'])" gpurun_out/b_${TAG}.json
