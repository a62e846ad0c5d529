# FAST dynamic-LDS padding sweep (fewer FAST workgroups per CU leave room for the latency-bound kernels of the
# other pipelined batches); needs a library built with the ORBX_FAST_PAD experiment hook
set -o pipefail
cd $GRAFT_REPO_ROOT
for i in 1 2; do
for PAD in 0 1500 2400 4000; do
  ORBX_FAST_PAD=$PAD timeout -k 10 300 python bench.py --no-cpu --host-steps 0 > gpurun_out/fpad.json 2>gpurun_out/fpad.err || { tail -20 gpurun_out/fpad.err; exit 1; }
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], d['value'], d['ms_per_step'], d['stage_ms_isolated']['fast'])" gpurun_out/fpad.json $PAD
done
done
