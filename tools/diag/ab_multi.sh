# A/B of the default liborbx.so against alternative builds (tools/diag/build_alt.sh), isolated stage times,
# two rounds in alternating order:  bash tools/diag/ab_multi.sh "DIR1 DIR2 ..." [bench args]
set -o pipefail
R=$GRAFT_REPO_ROOT
DIRS=$1; shift
cd $R
for i in 1 2; do
  for L in default $DIRS; do
    if [ $L = default ]; then unset ORBX_LIB; else export ORBX_LIB=$R/orb-slam-_amd/$L/liborbx.so; fi
    timeout -k 10 300 python bench.py --no-cpu --host-steps 0 --ingress-peers 0 --steps 20 --warmup 5 "$@" > gpurun_out/abl.json 2>gpurun_out/abl.err || exit 1
    python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], d['value'], d['ms_per_step'], d['stage_ms_isolated'])" gpurun_out/abl.json $L
  done
done
