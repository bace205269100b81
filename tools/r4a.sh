set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out/r4a
ok() { case $1 in 0|1) return 0;; *) echo "step ended with $1: stopping"; exit "$1";; esac; }   # 1 = test failures
timeout -k 10 300 python3 -u tools/grad_err_groups.py --out gpurun_out/r4a/grad_groups.json > gpurun_out/r4a/grad_groups.log 2>&1 || exit $?
STEPS=3 bash tools/gpu.sh trace r4a_t512 512 > gpurun_out/r4a/t512.txt 2>&1 || exit $?
STEPS=3 bash tools/gpu.sh trace r4a_t512deep 512 PFR_LEAF_SIZE=10000 > gpurun_out/r4a/t512deep.txt 2>&1 || exit $?
FREQS=512 STEPS=6 bash tools/gpu.sh env r4a_ab512 "PFR_FLOW=0" "PFR_FLOW=3" "PFR_FLOW=7" "PFR_FLOW=7 PFR_LEAF_SIZE=10000" "PFR_FLOW=0" "PFR_FLOW=7" > gpurun_out/r4a/ab512.txt 2>&1 || exit $?
FREQS=2048 STEPS=3 bash tools/gpu.sh env r4a_ab2048 "PFR_FLOW=0 PFR_FUSE_ASM=0" "PFR_FLOW=0" "PFR_FLOW=3" "PFR_FLOW=7" "PFR_FLOW=0" > gpurun_out/r4a/ab2048.txt 2>&1 || exit $?
PFR_TEST_REPORT=gpurun_out/r4a/flow_report.jsonl timeout -k 10 700 python3 -u -m pytest tests/test_gpu_flow.py tests/test_gpu_hessian.py -m gpu -v --timeout 300 --timeout-method thread -k "flow or hessian_matches" > gpurun_out/r4a/flow_tests.log 2>&1; ok $?
timeout -k 10 300 python3 -u tools/grad_err_groups.py --check 15 --out gpurun_out/r4a/grad_groups_refine.json > gpurun_out/r4a/grad_groups_refine.log 2>&1 || exit $?
