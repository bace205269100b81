# Kernel trace of the default bench (two lanes) for GPU-idle analysis: bash tools/gpu_trace_default.sh OUT
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:-trace_default}
mkdir -p $O
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O -o run -- python3 bench.py --no-cpu-baseline --steps 3 --warmup 1 > $O/bench.json 2> $O/trace.err && echo DONE
