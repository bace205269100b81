# Round measurement on one MI355X: GPU tests, PMC traffic passes (lanes = 1), the default bench
# (reads the fresh traffic), and a rocprofv3 kernel-trace --stats profile of the bench with lanes = 1
# and 2,048-frequency chunks (so per-launch durations are those of the isolated sweep the bench roofline uses).
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:-round}
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/gpu_tests.log 2>&1 || { tail -30 $O/gpu_tests.log; exit 1; }
tail -2 $O/gpu_tests.log
PFR_LANES=1 timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d $O/fetch -o run -- python3 bench.py --steps 1 --warmup 0 --freqs 2048 --no-cpu-baseline > $O/fetch.json 2> $O/fetch.err || exit 1
PFR_LANES=1 timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d $O/write -o run -- python3 bench.py --steps 1 --warmup 0 --freqs 2048 --no-cpu-baseline > $O/write.json 2> $O/write.err || exit 1
python3 tools/pmc_summary.py $O/fetch $O/write --last-sweep --freqs 2048 --json $O/pmc_traffic.json \
  --note "rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE (separate passes) --kernel-trace of: PFR_LANES=1 python bench.py --steps 1 --warmup 0 --freqs 2048 --no-cpu-baseline; last sweep (timed step + isolated sweep)" > $O/pmc_summary.txt || exit 1
cp $O/pmc_traffic.json profiles/r01/pmc_traffic.json
timeout -k 10 400 python -u bench.py > $O/bench.json 2> $O/bench.err || exit 1
cat $O/bench.json
PFR_LANES=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/stats -o run -- python3 bench.py --no-cpu-baseline --chunk 2048 > $O/bench_prof_l1.json 2> $O/stats.err || exit 1
echo DONE
