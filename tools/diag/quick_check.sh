# One-box check of a kernel change: the parity/fuzz/golden/caps GPU tests, one-stream kernel times,
# FETCH_SIZE of the FAST and quadtree kernels, and two pipelined bench lines.
#   bash tools/diag/quick_check.sh TAG
set -o pipefail
R=$GRAFT_REPO_ROOT
TAG=${1:-qc}
cd $R
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fuzz.py tests/test_golden.py tests/test_caps.py -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/pt_$TAG.log 2>&1 || { tail -30 gpurun_out/pt_$TAG.log; exit 1; }
tail -1 gpurun_out/pt_$TAG.log
bash tools/diag/kstats.sh $TAG > gpurun_out/ks_$TAG.txt || exit 1
head -12 gpurun_out/ks_$TAG.txt
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $R/gpurun_out/fetch_$TAG -o run -- python3 $R/bench.py --steps 3 --warmup 1 --no-cpu --streams 1 --iso-steps 0 --host-steps 0 > /dev/null 2>&1 || { echo FETCH_FAIL; exit 1; }
python3 - $R/gpurun_out/fetch_$TAG <<'PY'
import csv, glob, sys, collections
d = collections.defaultdict(list)
for fn in glob.glob(sys.argv[1] + "/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(fn)):
        n = r["Kernel_Name"].split("(")[0]
        if "qt_" in n or "quadtree" in n or "fast" in n or "describe" in n:
            d[n].append(float(r["Counter_Value"]))
for k, v in sorted(d.items()):
    print("%-40s fetch %.1f MB x2 (corrected)" % (k.split("::")[-1], 2 * sum(v) / len(v) / 1024))
PY
cd $R
for i in 1 2; do
  timeout -k 10 300 python bench.py --no-cpu --host-steps 0 --iso-steps 0 > gpurun_out/b_${TAG}_$i.json 2>gpurun_out/b_${TAG}_$i.err || { tail -5 gpurun_out/b_${TAG}_$i.err; exit 1; }
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print('bench', d['value'], d['ms_per_step'])" gpurun_out/b_${TAG}_$i.json
done
