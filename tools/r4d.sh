set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
O=gpurun_out/r4d
mkdir -p $O
ok() { case $1 in 0|1) return 0;; *) echo "step ended with $1: stopping"; exit "$1";; esac; }
timeout -k 10 300 python3 -u tools/grad_err_groups.py --check 11 --out $O/g11.json > $O/g11.log 2>&1 || exit $?
timeout -k 10 300 python3 -u tools/grad_err_groups.py --check 27 --out $O/g27.json > $O/g27.log 2>&1 || exit $?
PFR_SCALE_CORR=0 timeout -k 10 300 python3 -u tools/grad_err_groups.py --check 11 --out $O/g11_noscale.json > $O/g11_noscale.log 2>&1 || exit $?
FREQS=4096 STEPS=4 bash tools/gpu.sh env r4d_ab4096 "PFR_CHECK=11" "PFR_CHECK=11 PFR_SCALE_CORR=0" "PFR_CHECK=27" > $O/ab4096.txt 2>&1 || exit $?
PFR_CHECK=11 PFR_TEST_REPORT=$O/test_report.jsonl timeout -k 10 600 python3 -u -m pytest tests/test_gpu_grad_truth.py tests/test_gpu_fullsize.py tests/test_gpu_c5.py -m gpu -v --timeout 300 --timeout-method thread > $O/tests.log 2>&1; ok $?
