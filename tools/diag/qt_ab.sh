# Path-code quadtree against the node-list kernel (default; the path kernel with ORBX_QT_PATHS=1) on one box: one-stream kernel times of
# each, FETCH_SIZE of the quadtree kernels of each, and alternating pipelined bench lines.
#   bash tools/diag/qt_ab.sh TAG
set -o pipefail
R=$GRAFT_REPO_ROOT
TAG=${1:-qab}
cd $R
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fuzz.py -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/pt_$TAG.log 2>&1 || { tail -30 gpurun_out/pt_$TAG.log; exit 1; }
ORBX_QT_PATHS=1 timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fuzz.py -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/pt_${TAG}_nodes.log 2>&1 || { tail -30 gpurun_out/pt_${TAG}_nodes.log; exit 1; }
tail -1 gpurun_out/pt_$TAG.log gpurun_out/pt_${TAG}_nodes.log
ORBX_QT_PATHS=1 bash tools/diag/kstats.sh ${TAG}_p > gpurun_out/ks_${TAG}_p.txt || exit 1
bash tools/diag/kstats.sh ${TAG}_n > gpurun_out/ks_${TAG}_n.txt || exit 1
grep -E "qt_|quadtree" gpurun_out/ks_${TAG}_p.txt | head -6; grep -E "qt_|quadtree" gpurun_out/ks_${TAG}_n.txt | head -3
cd /tmp && export TMPDIR=/tmp
for M in p n; do
  if [ $M = p ]; then export ORBX_QT_PATHS=1; else unset ORBX_QT_PATHS; fi
  timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $R/gpurun_out/fetch_${TAG}_$M -o run -- python3 $R/bench.py --steps 3 --warmup 1 --no-cpu --streams 1 --iso-steps 0 --host-steps 0 > /dev/null 2>&1 || { echo FETCH_FAIL; exit 1; }
  python3 - $R/gpurun_out/fetch_${TAG}_$M $M <<'PY'
import csv, glob, sys, collections
d = collections.defaultdict(list)
for fn in glob.glob(sys.argv[1] + "/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(fn)):
        n = r["Kernel_Name"].split("(")[0]
        if "qt_" in n or "quadtree" in n:
            d[n].append(float(r["Counter_Value"]))
for k, v in sorted(d.items()):
    print(sys.argv[2], "%-40s fetch %.1f MB x2 (corrected)" % (k.split("::")[-1], 2 * sum(v) / len(v) / 1024))
PY
done
cd $R
for i in 1 2; do
  for M in p n; do
    if [ $M = p ]; then export ORBX_QT_PATHS=1; else unset ORBX_QT_PATHS; fi
    timeout -k 10 300 python bench.py --no-cpu --host-steps 0 --iso-steps 0 > gpurun_out/b_${TAG}_$M.json 2>gpurun_out/b_${TAG}_$M.err || { tail -5 gpurun_out/b_${TAG}_$M.err; exit 1; }
    python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], d['value'], d['ms_per_step'])" gpurun_out/b_${TAG}_$M.json $M
  done
done
