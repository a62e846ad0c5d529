set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fuzz.py tests/test_gpu_init.py -x -q --timeout 120 --timeout-method thread > gpurun_out/pt_fast2.log 2>&1 || { tail -30 gpurun_out/pt_fast2.log; exit 1; }
tail -1 gpurun_out/pt_fast2.log
timeout -k 10 200 python bench.py --no-cpu --host-steps 0 > gpurun_out/b_fast2.json 2> gpurun_out/b_fast2.err || { tail gpurun_out/b_fast2.err; exit 1; }
python3 -c "import json; d=json.load(open('gpurun_out/b_fast2.json')); print(d['value'], d['stage_ms_isolated'])"
timeout -k 10 120 python3 tools/diag/fast_prof.py build_fprof
