# one-stream kernel averages (tools/diag/kstats.sh) of the default library and alternative builds
#   bash tools/diag/kstats_alts.sh PATTERN DIR1 [DIR2 ...]
set -o pipefail
R=$GRAFT_REPO_ROOT
K=$1; shift
for L in default "$@"; do
  if [ $L = default ]; then unset ORBX_LIB; else export ORBX_LIB=$R/orb-slam-_amd/$L/liborbx.so; fi
  bash $R/tools/diag/kstats.sh ka_$L > $R/gpurun_out/ka_$L.txt || exit 1
  echo "$L: $(grep -E "$K" $R/gpurun_out/ka_$L.txt | head -3 | tr -s ' ' | tr '\n' ';')"
done
