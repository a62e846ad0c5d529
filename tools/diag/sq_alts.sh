# SQ counters (tools/gpu_sq.sh) of the extract kernels for the default library and alternative builds
#   bash tools/diag/sq_alts.sh DIR1 [DIR2 ...]
set -o pipefail
R=$GRAFT_REPO_ROOT
for L in default "$@"; do
  if [ $L = default ]; then unset ORBX_LIB; else export ORBX_LIB=$R/orb-slam-_amd/$L/liborbx.so; fi
  echo "== $L"
  bash $R/tools/gpu_sq.sh sqa_$L > $R/gpurun_out/sqa_$L.txt 2>&1 || { tail -5 $R/gpurun_out/sqa_$L.txt; exit 1; }
  grep -A1 -E "k_fast|k_describe" $R/gpurun_out/sqa_$L.txt
done
