# SQ counters of k_describe (or any kernel) for the default build and alternative builds, one pass each:
#   bash tools/diag/sq_ab.sh "DIR1 DIR2" [counter list]   (rows of tools/sq_summary.py for k_describe)
set -o pipefail
R=$GRAFT_REPO_ROOT
DIRS=$1
C=${2:-"SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU"}
cd /tmp && export TMPDIR=/tmp
for L in default $DIRS; do
  if [ $L = default ]; then unset ORBX_LIB; else export ORBX_LIB=$R/orb-slam-_amd/$L/liborbx.so; fi
  rm -rf $R/gpurun_out/sqab_$L
  timeout -s KILL 120 rocprofv3 --pmc $C --output-format csv -d $R/gpurun_out/sqab_$L -o run -- python3 $R/bench.py --steps 2 --warmup 1 --no-cpu --streams 1 --iso-steps 0 --host-steps 0 --ingress-peers 0 > $R/gpurun_out/sqab_$L.json 2> $R/gpurun_out/sqab_$L.err || { echo SQ_FAIL $L; tail -5 $R/gpurun_out/sqab_$L.err; exit 1; }
  echo "== $L"; python3 $R/tools/sq_summary.py $R/gpurun_out/sqab_$L | grep -A1 "^k_describe"
done
