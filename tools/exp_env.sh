# Kernel-class times (one isolated 2048-frequency chunk) for several environment settings:
#   bash tools/exp_env.sh "PFR_LANES=1 PFR_SCHUR_PF=0" "PFR_LANES=1 PFR_SCHUR_PF=1" ...
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/exp
i=0
for cfg in "$@"; do
  i=$((i+1))
  env $cfg timeout -k 10 200 python -u bench.py --no-cpu-baseline --steps 3 --freqs ${FREQS:-2048} > gpurun_out/exp/e$i.json 2> gpurun_out/exp/e$i.err || { tail -5 gpurun_out/exp/e$i.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/exp/e$i.json'));f=d['factor_roofline'];p=d['phase_ms'];print('$cfg |', round(d['value']), [round(x,2) for x in f['ms']], {k:round(v,2) for k,v in p.items() if k!='note'})"
done
