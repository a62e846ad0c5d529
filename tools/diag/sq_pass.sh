# one extra SQ counter pass (at most 8 SQ_ counters) over one-stream bench steps, per-kernel averages
#   bash tools/diag/sq_pass.sh TAG COUNTER...
set -o pipefail
R=$GRAFT_REPO_ROOT
TAG=$1; shift
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --pmc "$@" --output-format csv -d $R/gpurun_out/$TAG -o run -- python3 $R/bench.py --steps 3 --warmup 1 --no-cpu --streams 1 --iso-steps 0 --host-steps 0 > $R/gpurun_out/$TAG.json 2> $R/gpurun_out/$TAG.err || { echo SQ_FAIL; tail -20 $R/gpurun_out/$TAG.err; exit 1; }
python3 $R/tools/sq_summary.py $R/gpurun_out/$TAG
