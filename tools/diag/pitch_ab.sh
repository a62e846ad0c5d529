set -o pipefail
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp
mkdir -p gpurun_out/pitch
rm -rf gpurun_out/pitch; mkdir -p gpurun_out/pitch
for p in 0 1248; do
  timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/pitch/p$p -o run -- python3 tools/diag/pitch_ab.py --pad $p > gpurun_out/pitch/p$p.err 2>&1 || exit 1; grep -E "pitch|==" gpurun_out/pitch/p$p.err
done
for p in 0 1248; do echo "== pad $p"; f=$(ls gpurun_out/pitch/p$p/*/run_kernel_stats.csv 2>/dev/null || ls gpurun_out/pitch/p$p/run_kernel_stats.csv); python3 -c "
import csv,sys
for r in csv.DictReader(open('$f')):
    print('%-45s %8.1f us x %s' % (r['Name'][:45], float(r['AverageNs'])/1e3, r['Calls']))
"; done
