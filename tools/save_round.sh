# Copy one gpu_round.sh result (gpurun_out/round_TAG) into profiles/RND as version V:
#   bash tools/save_round.sh TAG RND V
set -e
T=${1:?tag}; RND=${2:?round dir}; V=${3:?version}
S=gpurun_out/round_$T; D=profiles/$RND
mkdir -p $D
cp $S/bench.json $D/bench_$V.json
cp $S/prof/run_kernel_stats.csv $D/bench_kernel_stats_$V.csv
cp $S/prof_pipelined/run_kernel_stats.csv $D/bench_kernel_stats_${V}_pipelined.csv
cp $S/sq.txt $D/sq_$V.txt
cp $S/pmc_traffic.json $D/pmc_traffic_$V.json
cp $S/pytest_gpu.log $D/pytest_gpu_$V.log
cp $S/smoke.log $D/smoke_$V.log
# the counter files bench.py reads (it reports their figures only for its own batch and kernel sources)
cp $S/pmc_traffic.json profiles/pmc_traffic.json
cp $S/sq_counters.json profiles/sq_counters.json
