# rocprofv3 kernel-trace --stats of one lanes=1 bench run in 2,048-frequency chunks (per-kernel,
# per-level durations of isolated launches): bash tools/gpu_stats.sh OUTNAME
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:-stats}
mkdir -p $O
PFR_LANES=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O -o run -- python3 bench.py --no-cpu-baseline --chunk 2048 --steps 2 --warmup 1 > $O/bench.json 2> $O/stats.err && echo DONE
