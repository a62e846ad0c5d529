# HBM traffic of the bench's kernels from rocprofv3 PMC counters, one counter per pass
# (MI355X_MICROARCH.md "HBM": FETCH_SIZE and WRITE_SIZE cannot share a pass; no sys/runtime trace).
#   bash tools/collect_pmc.sh TAG     (on the GPU box) -> gpurun_out/pmc_TAG/{fetch,write}/...
set -o pipefail
R=$GRAFT_REPO_ROOT
TAG=${1:-r01}
cd /tmp && export TMPDIR=/tmp
mkdir -p $R/gpurun_out/pmc_$TAG
for C in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 300 rocprofv3 --pmc $C --output-format csv -d $R/gpurun_out/pmc_$TAG/$C -o run -- \
    python3 $R/bench.py --steps 5 --warmup 1 --no-cpu --host-steps 0 > $R/gpurun_out/pmc_$TAG/bench_$C.json 2> $R/gpurun_out/pmc_$TAG/bench_$C.err \
    || { echo PMC_FAIL $C; tail -20 $R/gpurun_out/pmc_$TAG/bench_$C.err; exit 1; }
done
python3 $R/tools/pmc_summary.py $R/gpurun_out/pmc_$TAG --profiles $R/gpurun_out/pmc_$TAG/pmc_traffic.json
