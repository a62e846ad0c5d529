set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fuzz.py tests/test_gpu_init.py -x -q --timeout 120 --timeout-method thread > gpurun_out/pt_fast3.log 2>&1 || { tail -30 gpurun_out/pt_fast3.log; exit 1; }
tail -1 gpurun_out/pt_fast3.log
bash tools/diag/kstats_alts.sh "k_fast|k_describe|k_si" build_desc0 build_oldfast || exit 1
timeout -k 10 200 python bench.py --no-cpu --host-steps 0 > gpurun_out/b_fast3.json 2> gpurun_out/b_fast3.err || { tail gpurun_out/b_fast3.err; exit 1; }
python3 -c "import json; d=json.load(open('gpurun_out/b_fast3.json')); print(d['value'], d['stage_ms_isolated'])"
