# Profiles of one bench run (lanes = 1 so per-launch durations are not shared with a second lane):
# kernel-trace stats, then FETCH_SIZE and WRITE_SIZE in separate --pmc passes.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:-prof}
mkdir -p $O
export PFR_LANES=1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/stats -o run -- python3 bench.py --no-cpu-baseline --steps 2 --warmup 1 > $O/bench_l1.json 2> $O/stats.err && \
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d $O/fetch -o run -- python3 bench.py --steps 1 --warmup 0 --freqs 2048 --no-cpu-baseline > $O/fetch.json 2> $O/fetch.err && \
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d $O/write -o run -- python3 bench.py --steps 1 --warmup 0 --freqs 2048 --no-cpu-baseline > $O/write.json 2> $O/write.err
echo DONE $?
