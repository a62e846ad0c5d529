# per-launch-shape kernel times (one stream) + one bench line with the copy probe
set -o pipefail
R=$GRAFT_REPO_ROOT
TAG=${1:-k}
cd $R
bash tools/diag/kstats.sh $TAG > gpurun_out/ks_$TAG.txt 2>&1 || { tail -20 gpurun_out/ks_$TAG.txt; exit 1; }
cat gpurun_out/ks_$TAG.txt
cd $R
timeout -k 10 300 python bench.py --no-cpu --host-steps 0 --steps 20 --warmup 5 > gpurun_out/b_$TAG.json 2> gpurun_out/b_$TAG.err || { tail -20 gpurun_out/b_$TAG.err; exit 1; }
python3 -c "import json; d=json.load(open('gpurun_out/b_$TAG.json')); print(d['value'], d['ms_per_step'], d['stage_ms_isolated']); print(d['roofline'].get('hbm_copy'))"
