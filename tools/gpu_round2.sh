# Round measurement on one MI355X (round directory R, default r02):
#   1. every GPU test (per-test report), 2. PMC FETCH_SIZE / WRITE_SIZE passes (lanes = 1, one
#   2,048-frequency step) -> pmc_traffic.json, 3. the default bench (reads the fresh traffic when it
#   has been copied to profiles/R), 4. rocprofv3 --kernel-trace --stats of the bench with lanes = 1
#   and 2,048-frequency chunks, 5. the C5 L-BFGS run (tools/c5_lbfgs.py).
# Stops at the first GPU fault / abort / timeout (124, 134, 137, 139).
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
R=${1:-r02}
O=gpurun_out/$R
mkdir -p $O
stop() { case $1 in 124|134|137|139) echo "step ended with $1: stopping"; exit $1;; esac; }
PFR_TEST_REPORT=$O/test_report.jsonl timeout -k 10 1000 python -u -m pytest tests -m gpu -v --timeout 300 \
  --timeout-method thread > $O/gpu_tests.log 2>&1
rc=$?; tail -3 $O/gpu_tests.log; stop $rc
PFR_LANES=1 timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d $O/fetch -o run -- python3 bench.py --steps 1 --warmup 0 --freqs 2048 --no-cpu-baseline > $O/fetch.json 2> $O/fetch.err || exit $?
PFR_LANES=1 timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d $O/write -o run -- python3 bench.py --steps 1 --warmup 0 --freqs 2048 --no-cpu-baseline > $O/write.json 2> $O/write.err || exit $?
python3 tools/pmc_summary.py $O/fetch $O/write --last-sweep --freqs 2048 --json $O/pmc_traffic.json \
  --note "rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE (separate passes) --kernel-trace of: PFR_LANES=1 python bench.py --steps 1 --warmup 0 --freqs 2048 --no-cpu-baseline; last sweep (timed step + isolated sweep)" > $O/pmc_summary.txt || exit 1
mkdir -p profiles/$R && cp $O/pmc_traffic.json profiles/$R/pmc_traffic.json
timeout -k 10 400 python -u bench.py > $O/bench.json 2> $O/bench.err || exit $?
cat $O/bench.json
PFR_LANES=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/stats -o run -- python3 bench.py --no-cpu-baseline --chunk 2048 > $O/bench_prof_l1.json 2> $O/stats.err || exit $?
timeout -k 10 600 python -u tools/c5_lbfgs.py > $O/c5.json 2> $O/c5.err || exit $?
cat $O/c5.json
[ $rc -ne 0 ] && exit $rc
echo DONE
