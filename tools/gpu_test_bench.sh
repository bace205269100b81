# GPU tests then one bench run (each step under its own time limit; stop at the first failure)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
PFR_TEST_REPORT=$GRAFT_REPO_ROOT/gpurun_out/test_report.jsonl timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread ${PYTEST_K:+-k "$PYTEST_K"} > gpurun_out/gpu_tests.log 2>&1 && \
timeout -k 10 300 python -u bench.py ${BENCH_ARGS:---no-cpu-baseline} > gpurun_out/bench.json 2> gpurun_out/bench.err
rc=$?
tail -3 gpurun_out/gpu_tests.log
cat gpurun_out/bench.json
exit $rc
