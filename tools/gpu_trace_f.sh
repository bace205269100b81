# Per-level kernel times of one lanes=1 bench step at F frequencies in one chunk:
#   bash tools/gpu_trace_f.sh OUT F
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp PFR_LANES=1
O=gpurun_out/${1:-tracef}
F=${2:-4096}
mkdir -p $O
timeout -k 10 240 rocprofv3 --kernel-trace --output-format csv -d $O -o run -- python3 bench.py --steps 1 --warmup 0 --freqs $F --chunk $F --no-cpu-baseline > $O/b.json 2> $O/err || exit 1
python3 tools/level_times.py $O/run_kernel_trace.csv
