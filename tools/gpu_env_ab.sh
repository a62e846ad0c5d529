# A/B of library environment knobs: GPU parity tests on the default, then alternating no-CPU bench
# lines per variant (each variant a space-separated list of VAR=value, "-" for the default), two rounds.
#   bash tools/gpu_env_ab.sh TAG "-" "ORBX_PYR_NARROW=0" ...
set -o pipefail
R=$GRAFT_REPO_ROOT
TAG=${1:-env}
shift
O=$R/gpurun_out/env_$TAG
mkdir -p $O
cd $R
timeout -k 10 300 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for round in 1 2; do
  i=0
  for v in "$@"; do
    i=$((i + 1))
    envs=""
    [ "$v" != "-" ] && envs="$v"
    f=$O/b_${i}_$round.json
    env $envs timeout -k 10 200 python bench.py --no-cpu --host-steps 0 > $f 2> $O/b.err || { tail -20 $O/b.err; exit 1; }
    python3 -c "import json; d=json.load(open('$f')); print('[$v] r$round', d['value'], {k: round(x, 4) for k, x in d['stage_ms_isolated'].items()})"
  done
done
