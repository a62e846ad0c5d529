# LDS bank-conflict attribution: LDS counters and one-stream kernel times of the default library and
# diagnostic builds (tools/diag/build_alt.sh DIR -DORBX_DIAG_*_LIN; their results are wrong by design)
#   bash tools/diag/lds_attr.sh KERNEL DIR1 [DIR2 ...]
set -o pipefail
R=$GRAFT_REPO_ROOT
K=$1; shift
for L in default "$@"; do
  if [ $L = default ]; then unset ORBX_LIB; else export ORBX_LIB=$R/orb-slam-_amd/$L/liborbx.so; fi
  echo "== $L"
  bash $R/tools/diag/sq_pass.sh lds_$L SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_WAIT_INST_LDS > $R/gpurun_out/lds_$L.txt 2>&1 || { tail -5 $R/gpurun_out/lds_$L.txt; exit 1; }
  grep -E "^$K" $R/gpurun_out/lds_$L.txt
  bash $R/tools/diag/kstats.sh lk_$L | grep -E "$K" | head -2
done
