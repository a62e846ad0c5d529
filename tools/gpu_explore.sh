# Exploration run: parity tests, bench at several batch sizes, SQ instruction-mix counters.
set -o pipefail
R=$GRAFT_REPO_ROOT
TAG=${1:-x}
cd $R
timeout -k 10 900 python -m pytest tests -x -q -m gpu > gpurun_out/pytest_gpu_$TAG.log 2>&1 || { echo PYTEST_FAIL; tail -40 gpurun_out/pytest_gpu_$TAG.log; exit 1; }
tail -1 gpurun_out/pytest_gpu_$TAG.log
for B in 64 128 256; do
  timeout -k 10 300 python bench.py --batch $B --no-cpu > gpurun_out/bench_${TAG}_b$B.json 2> gpurun_out/bench_${TAG}_b$B.err || { echo BENCH_FAIL $B; tail -20 gpurun_out/bench_${TAG}_b$B.err; exit 1; }
  python3 -c "import json,sys; d=json.load(open('gpurun_out/bench_${TAG}_b$B.json')); print($B, d['value'], d['stage_ms_per_step'])"
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_VALU SQ_LDS_BANK_CONFLICT --output-format csv -d $R/gpurun_out/sq_$TAG -o run -- python3 $R/bench.py --steps 3 --warmup 1 --no-cpu > $R/gpurun_out/sq_$TAG.json 2> $R/gpurun_out/sq_$TAG.err || { echo SQ_FAIL; tail -20 $R/gpurun_out/sq_$TAG.err; exit 1; }
echo done
