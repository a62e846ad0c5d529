# Pyramid launch-group variants (ORBX_PYR_SPLIT: first level of each launch; ORBX_PYR_BAND: rows of a
# group's last level per block; ORBX_PYR_NT, ORBX_PYR_SPLITROWS): GPU parity tests on the default, then a
# no-CPU bench line per variant ("split:band:nt:splitrows", nt 0 = the library's choice).
#   bash tools/gpu_pyr_variants.sh TAG [variant ...]
set -o pipefail
R=$GRAFT_REPO_ROOT
TAG=${1:-pv}
shift
O=$R/gpurun_out/pv_$TAG
mkdir -p $O
cd $R
timeout -k 10 300 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for v in "$@"; do
  IFS=: read sp bd nt srows <<< "$v"
  envs="ORBX_PYR_SPLIT=$sp ORBX_PYR_BAND=$bd ORBX_PYR_SPLITROWS=$srows"
  [ "$nt" != "0" ] && envs="$envs ORBX_PYR_NT=$nt"
  f=$O/b_${v//[,:]/_}.json
  env $envs timeout -k 10 200 python bench.py --no-cpu --host-steps 0 > $f 2> $O/b.err || { tail -20 $O/b.err; exit 1; }
  python3 -c "import json; d=json.load(open('$f')); print('$v', d['value'], 'pyr iso', d['stage_ms_isolated']['pyramid'])"
done
