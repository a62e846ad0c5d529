# One SQ counter pass (issue / wait / LDS breakdown) of one-stream bench steps, per kernel.
#   bash tools/diag/sq_pass2.sh TAG
set -o pipefail
R=$GRAFT_REPO_ROOT
TAG=${1:-sq2}
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE --output-format csv -d $R/gpurun_out/$TAG -o run -- python3 $R/bench.py --steps 3 --warmup 1 --no-cpu --streams 1 --iso-steps 0 --host-steps 0 > $R/gpurun_out/$TAG.json 2> $R/gpurun_out/$TAG.err || { echo SQ_FAIL; tail -20 $R/gpurun_out/$TAG.err; exit 1; }
python3 - $R/gpurun_out/$TAG <<'PY'
import csv, glob, os, sys
from collections import defaultdict
vals = defaultdict(lambda: defaultdict(list))
for fn in glob.glob(os.path.join(sys.argv[1], "**", "*counter_collection.csv"), recursive=True):
    for r in csv.DictReader(open(fn)):
        k = r["Kernel_Name"].split("(")[0].split("::")[-1]
        vals[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, c in sorted(vals.items()):
    if not k.startswith("k_"): continue
    a = {n: sum(v) / len(v) for n, v in c.items()}
    wc = a.get("SQ_WAVE_CYCLES", 1) or 1
    print("%-28s waves %8.0f  cyc/wave %7.0f  wait_any %.2f  wait_inst %.2f (lds %.2f)  active %.2f  lds_idx %.3g  bank_confl %.3g" % (
        k[:28], a.get("SQ_WAVES", 0), wc / max(a.get("SQ_WAVES", 1), 1), a.get("SQ_WAIT_ANY", 0) / wc,
        a.get("SQ_WAIT_INST_ANY", 0) / wc, a.get("SQ_WAIT_INST_LDS", 0) / wc, a.get("SQ_ACTIVE_INST_ANY", 0) / wc,
        a.get("SQ_LDS_IDX_ACTIVE", 0), a.get("SQ_LDS_BANK_CONFLICT", 0)))
PY
