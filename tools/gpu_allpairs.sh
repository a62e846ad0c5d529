# all-pairs parity + config 5 (FULL_U16 / TOP2 timings)
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q -m gpu -k allpairs --timeout 120 --timeout-method thread 2>&1 | tail -2 || exit 1
timeout -k 10 300 python tools/bench_configs.py --config 5 > gpurun_out/cfg5.json 2> gpurun_out/cfg5.err || { tail -20 gpurun_out/cfg5.err; exit 1; }
python3 -c "import json; d=json.load(open('gpurun_out/cfg5.json')); print(d['full_u16_ms'], d['full_u16_roofline']['frac'], d['top2_ms'], d['extract_frames_per_s'])"
