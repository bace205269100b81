# Kernel-class times of one isolated chunk for several chunk sizes and both factorisation modes
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/exp
export PFR_LANES=1
for sym in 1 0; do for ch in 2048 512; do
  PFR_SYMMETRIC=$sym timeout -k 10 200 python -u bench.py --no-cpu-baseline --steps 2 --freqs 2048 --chunk $ch > gpurun_out/exp/s${sym}_c${ch}.json 2> gpurun_out/exp/s${sym}_c${ch}.err || exit 1
  python -c "import json;d=json.load(open('gpurun_out/exp/s${sym}_c${ch}.json'));f=d['factor_roofline'];print('sym=$sym chunk=$ch', round(d['value']), [round(x*2048/f['frequencies'],2) for x in f['ms']], d['phase_ms'])"
done; done
