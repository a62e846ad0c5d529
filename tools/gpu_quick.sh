# Quick loop: GPU parity tests, SQ counters of the extract kernels, a no-CPU bench line.
set -o pipefail
R=$GRAFT_REPO_ROOT
TAG=${1:-q}
cd $R
timeout -k 10 300 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/pt_$TAG.log 2>&1 || { tail -30 gpurun_out/pt_$TAG.log; exit 1; }
tail -1 gpurun_out/pt_$TAG.log
bash tools/gpu_sq.sh sq_$TAG | grep -A1 -E "k_fast|k_describe|k_quadtree|k_pyramid" || exit 1
cd $R
timeout -k 10 200 python bench.py --no-cpu > gpurun_out/b_$TAG.json 2>gpurun_out/b_$TAG.err || { tail -20 gpurun_out/b_$TAG.err; exit 1; }
python3 -c "import json; d=json.load(open('gpurun_out/b_$TAG.json')); print(d['value'], d['stage_ms_isolated'])"
