# SQ-mix and LDS counter passes for the extraction kernels, per alternative library (ORBX_LIB; "default" = the
# in-tree liborbx.so):   bash tools/r5/diaglibs.sh TAG LIB1 [LIB2 ...]
set -o pipefail
R=$GRAFT_REPO_ROOT
TAG=$1; shift
cd /tmp && export TMPDIR=/tmp
for L in "$@"; do
  if [ $L = default ]; then unset ORBX_LIB; else export ORBX_LIB=$R/orb-slam-_amd/$L/liborbx.so; fi
  O=$R/gpurun_out/r5dl_${TAG}_$L
  mkdir -p $O
  for P in "sq SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU" \
           "lds SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_INST_CYCLES_VMEM_RD"; do
    set -- $P; N=$1; shift
    timeout -s KILL 120 rocprofv3 --pmc "$@" --output-format csv -d $O/$N -o run -- python3 $R/bench.py --steps 3 --warmup 1 --no-cpu --streams 1 --iso-steps 0 --host-steps 0 --batch 1024 > $O/$N.json 2> $O/$N.err || { echo PMC_FAIL $L $N; tail -20 $O/$N.err; exit 1; }
    echo "== $L $N"; python3 $R/tools/sq_summary.py $O/$N | grep -E "k_describe|k_fast" -A1
  done
done
