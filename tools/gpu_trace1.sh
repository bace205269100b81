# One lanes=1 bench step at 2,048 frequencies under rocprofv3 --kernel-trace, then per-level times:
#   bash tools/gpu_trace1.sh OUT [ENV=V ...]
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp PFR_LANES=1
O=gpurun_out/${1:-trace1}
shift
mkdir -p $O
env "$@" timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $O -o run -- python3 bench.py --steps 1 --warmup 0 --freqs 2048 --no-cpu-baseline > $O/b.json 2> $O/err || exit 1
python3 tools/level_times.py $O/run_kernel_trace.csv
