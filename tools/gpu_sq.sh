# SQ instruction-mix / wait counters per kernel for one-stream bench steps.
set -o pipefail
R=$GRAFT_REPO_ROOT
TAG=${1:-sq}
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU --output-format csv -d $R/gpurun_out/$TAG -o run -- python3 $R/bench.py --steps 3 --warmup 1 --no-cpu --streams 1 --iso-steps 0 --host-steps 0 > $R/gpurun_out/$TAG.json 2> $R/gpurun_out/$TAG.err || { echo SQ_FAIL; tail -20 $R/gpurun_out/$TAG.err; exit 1; }
python3 $R/tools/sq_summary.py $R/gpurun_out/$TAG --save $R/gpurun_out/$TAG/sq_counters.json
