set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out/r4a
bash tools/gpu.sh tests r4a tests/test_gpu_grad_truth.py || exit $?
timeout -k 10 300 python3 -u tools/grad_err_groups.py --out gpurun_out/r4a/grad_groups.json > gpurun_out/r4a/grad_groups.log 2>&1 || exit $?
STEPS=3 bash tools/gpu.sh trace r4a_t512 512 || exit $?
STEPS=3 bash tools/gpu.sh trace r4a_t512deep 512 PFR_LEAF_SIZE=10000 || exit $?
FREQS=2048 STEPS=3 bash tools/gpu.sh env r4a_ab "PFR_FUSE_ASM=0" "PFR_FUSE_ASM=1" "PFR_FUSE_ASM=0" "PFR_FUSE_ASM=1" || exit $?
bash tools/gpu.sh tests r4a_flow tests/test_gpu_fullsize.py tests/test_gpu_flow.py || exit $?
FREQS=512 STEPS=6 bash tools/gpu.sh env r4a_ab512 "PFR_FLOW=0" "PFR_FLOW=1" "PFR_FLOW=3" "PFR_FLOW=7" "PFR_FLOW=7 PFR_LEAF_SIZE=10000" "PFR_FLOW=0" "PFR_FLOW=7" || exit $?
FREQS=2048 STEPS=3 bash tools/gpu.sh env r4a_ab2048 "PFR_FLOW=0" "PFR_FLOW=1" "PFR_FLOW=3" "PFR_FLOW=7" || exit $?
timeout -k 10 300 python3 -u tools/grad_err_groups.py --check 15 --out gpurun_out/r4a/grad_groups_refine.json > gpurun_out/r4a/grad_groups_refine.log 2>&1 || exit $?
