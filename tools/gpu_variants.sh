set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R
cp orb-slam-_amd/liborbx.so /tmp/base.so
for v in c2 c4 c6 base; do
  if [ $v = base ]; then cp /tmp/base.so orb-slam-_amd/liborbx.so; else cp orb-slam-_amd/variants/liborbx_$v.so orb-slam-_amd/liborbx.so; fi
  timeout -k 10 200 python bench.py --no-cpu > gpurun_out/var_$v.json 2>gpurun_out/var_$v.err || { tail -20 gpurun_out/var_$v.err; exit 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/var_$v.json')); print('$v', d['value'], d['stage_ms_isolated'])"
done
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q -m gpu --timeout 120 --timeout-method thread 2>&1 | tail -1
