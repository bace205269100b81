set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
O=gpurun_out/r4b
mkdir -p $O
ok() { case $1 in 0|1) return 0;; *) echo "step ended with $1: stopping"; exit "$1";; esac; }
timeout -k 10 300 python3 -u tools/grad_err_groups.py --out $O/grad_groups.json > $O/grad_groups.log 2>&1 || exit $?
PFR_REFINE_TOL=1e-7 timeout -k 10 300 python3 -u tools/grad_err_groups.py --out $O/grad_groups_tol1e-7.json > $O/grad_groups_tol1e-7.log 2>&1 || exit $?
FREQS=4096 STEPS=4 bash tools/gpu.sh env r4b_ab4096 "PFR_CHECK=11" "PFR_CHECK=27" "PFR_CHECK=11" "PFR_CHECK=27" "PFR_CHECK=27 PFR_REFINE_TOL=1e-7" > $O/ab4096.txt 2>&1 || exit $?
FREQS=512 STEPS=6 bash tools/gpu.sh env r4b_ab512 "PFR_CHECK=11" "PFR_CHECK=27" "PFR_MAX_NS=64" "PFR_MAX_NS=48" "PFR_MAX_NS=32" "PFR_LEAF_SIZE=10000 PFR_MAX_NS=64" "PFR_LEAF_SIZE=10000 PFR_MAX_NS=32" "PFR_LEAF_SIZE=500 PFR_MAX_NS=64" > $O/ab512.txt 2>&1 || exit $?
FREQS=4096 STEPS=4 bash tools/gpu.sh env r4b_ns4096 "PFR_MAX_NS=256" "PFR_MAX_NS=64" "PFR_MAX_NS=32" > $O/ns4096.txt 2>&1 || exit $?
FREQS=4096 STEPS=4 bash tools/gpu.sh env r4b_us2 "PFR_US2_CFG=0" "PFR_US2_CFG=1" "PFR_US2_CFG=2" "PFR_US2_CFG=0" > $O/us2.txt 2>&1 || exit $?
PFR_TEST_REPORT=$O/test_report.jsonl timeout -k 10 900 python3 -u -m pytest tests/test_gpu_grad_truth.py tests/test_gpu_fullsize.py tests/test_gpu_check.py tests/test_gpu_hessian.py tests/test_gpu_parity.py -m gpu -v --timeout 300 --timeout-method thread > $O/tests.log 2>&1; ok $?
