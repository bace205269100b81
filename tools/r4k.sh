set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
O=gpurun_out/r4k
mkdir -p $O
FREQS=512 STEPS=8 bash tools/gpu.sh env r4k_512 "PFR_LEAF_SIZE=96" "PFR_LEAF_SIZE=200" "PFR_LEAF_SIZE=300" "PFR_LEAF_SIZE=400" "PFR_LEAF_SIZE=700" "PFR_LEAF_SIZE=96" "PFR_LEAF_SIZE=300" > $O/leaf512.txt 2>&1 || exit $?
FREQS=1024 STEPS=6 bash tools/gpu.sh env r4k_1024 "PFR_LEAF_SIZE=10000" "PFR_LEAF_SIZE=300" "PFR_LEAF_SIZE=1000" "PFR_LEAF_SIZE=3000" "PFR_LEAF_SIZE=10000" > $O/leaf1024.txt 2>&1 || exit $?
FREQS=4096 STEPS=4 bash tools/gpu.sh env r4k_4096 "PFR_LEAF_SIZE=10000" "PFR_LEAF_SIZE=3000" "PFR_LEAF_SIZE=1000" "PFR_LEAF_SIZE=10000" > $O/leaf4096.txt 2>&1 || exit $?
