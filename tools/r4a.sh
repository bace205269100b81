set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out/r4a
bash tools/gpu.sh tests r4a tests/test_gpu_grad_truth.py tests/test_gpu_fullsize.py || exit $?
timeout -k 10 300 python3 -u tools/grad_err_groups.py --out gpurun_out/r4a/grad_groups.json > gpurun_out/r4a/grad_groups.log 2>&1 || exit $?
FREQS=2048 STEPS=3 bash tools/gpu.sh env r4a_fuse "PFR_FUSE_ASM=0" "PFR_FUSE_ASM=1" "PFR_FUSE_ASM=0" "PFR_FUSE_ASM=1" || exit $?
STEPS=3 bash tools/gpu.sh trace r4a_t512 512 || exit $?
STEPS=3 bash tools/gpu.sh trace r4a_t512deep 512 PFR_LEAF_SIZE=10000 || exit $?
timeout -k 10 300 python3 -u tools/grad_err_groups.py --check 15 --out gpurun_out/r4a/grad_groups_refine.json > gpurun_out/r4a/grad_groups_refine.log 2>&1 || exit $?
