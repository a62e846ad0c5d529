# FAST A/B on one GPU: SQ counters (one stream) and the phase profile of the current tree against an
# alternative build (default orb-slam-_amd/build_oldfast + build_oldfprof, tools/diag/build_alt.sh).
#   bash tools/diag/fast_ab.sh TAG [ALTDIR] [ALTPROFDIR]
set -o pipefail
R=$GRAFT_REPO_ROOT
TAG=${1:-fab}; ALT=${2:-build_oldfast}; ALTP=${3:-build_oldfprof}
cd /tmp && export TMPDIR=/tmp
SQ="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU"
for v in new alt; do
  if [ $v = alt ]; then export ORBX_LIB=$R/orb-slam-_amd/$ALT/liborbx.so; else unset ORBX_LIB; fi
  timeout -s KILL 120 rocprofv3 --pmc $SQ --output-format csv -d $R/gpurun_out/${TAG}_sq_$v -o run -- python3 $R/bench.py --steps 3 --warmup 1 --no-cpu --streams 1 --iso-steps 0 --host-steps 0 > $R/gpurun_out/${TAG}_sq_$v.json 2> $R/gpurun_out/${TAG}_sq_$v.err || { echo SQ_FAIL $v; tail -5 $R/gpurun_out/${TAG}_sq_$v.err; exit 1; }
  echo "== $v"; python3 $R/tools/sq_summary.py $R/gpurun_out/${TAG}_sq_$v | grep -A1 "k_fast"
done
unset ORBX_LIB
cd $R
echo "== new prof"; timeout -k 10 120 python3 tools/diag/fast_prof.py build_fprof || exit 1
echo "== alt prof"; timeout -k 10 120 python3 tools/diag/fast_prof.py $ALTP || exit 1
