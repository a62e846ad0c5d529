# Counter passes for the extraction kernels (one-stream bench steps): SQ mix, LDS conflicts, L2 hits, HBM fetch.
#   bash tools/r5/diag.sh TAG
set -o pipefail
R=$GRAFT_REPO_ROOT
TAG=${1:-d}
O=$R/gpurun_out/r5d_$TAG
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
run() {   # name, counters...
  local N=$1; shift
  timeout -s KILL 120 rocprofv3 --pmc "$@" --output-format csv -d $O/$N -o run -- python3 $R/bench.py --steps 3 --warmup 1 --no-cpu --streams 1 --iso-steps 0 --host-steps 0 --batch 1024 > $O/$N.json 2> $O/$N.err || { echo PMC_FAIL $N; tail -20 $O/$N.err; exit 1; }
  python3 $R/tools/sq_summary.py $O/$N | grep -E "k_describe|k_blur|k_fast|k_pyramid|k_quadtree" -A1
}
run sq SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU || exit 1
run lds SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR || exit 1
run tcc TCC_HIT_sum TCC_MISS_sum || exit 1
run fetch FETCH_SIZE || exit 1
