# FETCH_SIZE (x2, the gfx950 correction) per launch of the FAST, quadtree and describe kernels for the default
# library and alternative builds (tools/diag/build_alt.sh), one-stream bench steps.
#   bash tools/diag/fetch_libs.sh TAG [DIR ...]   (DIRs under orb-slam-_amd/)
set -o pipefail
R=$GRAFT_REPO_ROOT
TAG=$1; shift
cd /tmp && export TMPDIR=/tmp
for L in default "$@"; do
  if [ $L = default ]; then unset ORBX_LIB; else export ORBX_LIB=$R/orb-slam-_amd/$L/liborbx.so; fi
  timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $R/gpurun_out/fl_${TAG}_$L -o run -- python3 $R/bench.py --steps 3 --warmup 1 --no-cpu --streams 1 --iso-steps 0 --host-steps 0 > /dev/null 2>&1 || { echo FETCH_FAIL $L; exit 1; }
  python3 - $R/gpurun_out/fl_${TAG}_$L $L <<'PY'
import csv, glob, sys, collections
d = collections.defaultdict(list)
for fn in glob.glob(sys.argv[1] + "/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(fn)):
        n = r["Kernel_Name"].split("(")[0]
        if "qt_" in n or "quadtree" in n or "fast" in n or "describe" in n:
            d[n].append(float(r["Counter_Value"]))
tot = 0.0
for k, v in sorted(d.items()):
    mb = 2 * sum(v) / len(v) / 1024
    if "quadtree" in k or "qt_" in k:
        tot += mb
    print(sys.argv[2], "%-40s fetch %.1f MB" % (k.split("::")[-1], mb))
print(sys.argv[2], "quadtree launches together: %.1f MB" % tot)
PY
done
