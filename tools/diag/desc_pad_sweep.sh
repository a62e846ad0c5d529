set -o pipefail
cd $GRAFT_REPO_ROOT
export ORBX_LIB=$GRAFT_REPO_ROOT/orb-slam-_amd/build_alt_pad/liborbx.so
for PAD in 0 7000 15000 30000 0 7000 15000 30000; do
  ORBX_DESC_PAD=$PAD timeout -k 10 300 python bench.py --no-cpu --host-steps 0 > gpurun_out/pad.json 2>gpurun_out/pad.err || { tail -20 gpurun_out/pad.err; exit 1; }
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], d['value'], d['ms_per_step'], d['stage_ms_isolated'])" gpurun_out/pad.json $PAD
done
