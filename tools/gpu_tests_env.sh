# GPU tests under one environment setting (e.g. PFR_SCHUR_LDS=2), then exp_env.sh with the rest
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
env $1 timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1
rc=$?
tail -3 gpurun_out/gpu_tests.log
[ $rc -eq 0 ] || { grep -E "Error|error|assert" gpurun_out/gpu_tests.log | head -20; exit $rc; }
shift
bash tools/exp_env.sh "$@"
