set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
O=gpurun_out/r4x
mkdir -p $O
ok() { case $1 in 0|1) return 0;; *) echo "step ended with $1: stopping"; exit "$1";; esac; }
PFR_TEST_REPORT=$O/rep.jsonl timeout -k 10 400 python3 -u -m pytest tests/test_gpu_flow.py -k prefix -v --timeout 300 --timeout-method thread > $O/tests.log 2>&1; rc=$?; tail -3 $O/tests.log; ok $rc
[ $rc -eq 0 ] || exit 1
bash tools/gpu.sh trace r4x_t2048a 2048 PFR_OFF_PU=4 PFR_OFF_PU_WAVES=1000000000 > $O/t2048_pu4.txt 2>&1 || exit $?
bash tools/gpu.sh trace r4x_t2048b 2048 PFR_OFF_PU=8 PFR_OFF_PU_WAVES=1000000000 > $O/t2048_pu8.txt 2>&1 || exit $?
bash tools/gpu.sh trace r4x_t512a 512 PFR_OFF_PU=4 PFR_OFF_PU_WAVES=1000000000 > $O/t512_pu4.txt 2>&1 || exit $?
bash tools/gpu.sh trace r4x_t512b 512 PFR_OFF_PU=8 PFR_OFF_PU_WAVES=1000000000 > $O/t512_pu8.txt 2>&1 || exit $?
rm -f gpurun_out/r4x_t*/run_kernel_trace.csv
