# A/B of several alternative builds against the default library: extraction parity with each
# build, one-stream kernel averages, then alternating pipelined bench lines.
#   bash tools/diag/ab_multi.sh DIR1 [DIR2 ...]   (DIRs under orb-slam-_amd/, from tools/diag/build_alt.sh)
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
for L in default "$@"; do
  if [ $L = default ]; then unset ORBX_LIB; else export ORBX_LIB=$R/orb-slam-_amd/$L/liborbx.so; fi
  timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread > gpurun_out/abm_$L.log 2>&1 || { echo "PARITY FAIL $L"; tail -30 gpurun_out/abm_$L.log; exit 1; }
  echo "$L parity: $(tail -1 gpurun_out/abm_$L.log)"
  bash tools/diag/kstats.sh abm_$L > gpurun_out/abm_${L}_ks.txt || exit 1
  head -8 gpurun_out/abm_${L}_ks.txt
  cd $R
done
for i in $(seq 1 ${ABN:-2}); do
  for L in default "$@"; do
    if [ $L = default ]; then unset ORBX_LIB; else export ORBX_LIB=$R/orb-slam-_amd/$L/liborbx.so; fi
    timeout -k 10 300 python bench.py --no-cpu --host-steps 0 --iso-steps 0 > gpurun_out/abm.json || exit 1
    python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], d['value'], d['ms_per_step'])" gpurun_out/abm.json $L
  done
done
