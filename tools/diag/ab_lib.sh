# alternate pipelined bench runs of the default library and an alternative build
#   bash tools/diag/ab_lib.sh DIR [bench args]   (DIR under orb-slam-_amd/, from tools/diag/build_alt.sh)
set -o pipefail
R=$GRAFT_REPO_ROOT
D=$1; shift
cd $R
for i in 1 2; do
  for L in default $D; do
    if [ $L = default ]; then unset ORBX_LIB; else export ORBX_LIB=$R/orb-slam-_amd/$L/liborbx.so; fi
    timeout -k 10 300 python bench.py --no-cpu --host-steps 0 --iso-steps 0 "$@" > gpurun_out/abl.json || exit 1
    python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], d['value'], d['ms_per_step'])" gpurun_out/abl.json $L
  done
done
