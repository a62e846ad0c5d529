set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/prof_rows
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt -o run -- python3 $R/tools/bench_rows.py --cpu-seconds 0.2 > $O/kt.json 2> $O/kt.err || { echo KT_FAIL; tail $O/kt.err; exit 1; }
timeout -s KILL 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_INSTS_LDS --output-format csv -d $O/sq -o run -- python3 $R/tools/bench_rows.py --cpu-seconds 0.2 > $O/sq.json 2> $O/sq.err || { echo SQ_FAIL; tail $O/sq.err; exit 1; }
echo done
