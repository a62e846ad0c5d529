set -o pipefail
cd $GRAFT_REPO_ROOT
for B in 384 512 768 384 512 768; do
  timeout -k 10 300 python bench.py --no-cpu --host-steps 0 --iso-steps 0 --batch $B > gpurun_out/bs.json 2>gpurun_out/bs.err || { tail -20 gpurun_out/bs.err; exit 1; }
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], d['value'], d['ms_per_step'])" gpurun_out/bs.json $B
done
