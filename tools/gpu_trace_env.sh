# Kernel traces (lanes = 1, one 2048-frequency step) under several environment settings:
#   bash tools/gpu_trace_env.sh "PFR_SCHUR_LDS=0" "PFR_SCHUR_LDS=1" ...   -> gpurun_out/trace/tN/
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp PFR_LANES=1
i=0
for cfg in "$@"; do
  i=$((i+1))
  mkdir -p gpurun_out/trace/t$i
  echo "$cfg" > gpurun_out/trace/t$i/cfg
  env $cfg timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/trace/t$i -o run -- python3 bench.py --steps 1 --warmup 0 --freqs 2048 --no-cpu-baseline > gpurun_out/trace/t$i/b.json 2> gpurun_out/trace/t$i/err || exit 1
done
