# Full-size (4,096 frequencies) bench value for several lane / chunk settings:
#   bash tools/exp_lanes.sh "LANES CHUNK" ...   (CHUNK 0 = automatic)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/exp
i=0
for cfg in "$@"; do
  set -- $cfg
  i=$((i+1))
  extra=""; [ "$2" != "0" ] && extra="--chunk $2"
  PFR_LANES=$1 timeout -k 10 200 python -u bench.py --no-cpu-baseline --steps 5 $extra > gpurun_out/exp/l$i.json 2> gpurun_out/exp/l$i.err || { tail -5 gpurun_out/exp/l$i.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/exp/l$i.json'));print('lanes=$1 chunk=$2 |', round(d['value']), d['config']['chunk'], round(d['ms_per_step'],2))"
done
