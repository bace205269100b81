# Kernel-class times (one isolated 2048-frequency chunk, lanes = 1) in both factorisation modes
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/exp
export PFR_LANES=1
for sym in 1 0; do
  PFR_SYMMETRIC=$sym timeout -k 10 200 python -u bench.py --no-cpu-baseline --steps 2 --freqs 2048 > gpurun_out/exp/m${sym}.json 2> gpurun_out/exp/m${sym}.err || exit 1
  python -c "import json;d=json.load(open('gpurun_out/exp/m${sym}.json'));f=d['factor_roofline'];p=d['phase_ms'];print('sym=$sym', round(d['value']), [round(x,2) for x in f['ms']], {k:round(v,2) for k,v in p.items() if k!='note'})"
done
