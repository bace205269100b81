# GPU tests then one bench run (each step under its own time limit; stop at the first failure)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread ${PYTEST_K:+-k "$PYTEST_K"} > gpurun_out/gpu_tests.log 2>&1 && \
timeout -k 10 300 python -u bench.py ${BENCH_ARGS:---no-cpu-baseline} > gpurun_out/bench.json 2> gpurun_out/bench.err
rc=$?
tail -3 gpurun_out/gpu_tests.log
cat gpurun_out/bench.json
exit $rc
