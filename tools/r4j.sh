set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
O=gpurun_out/r4j
mkdir -p $O
FREQS=2048 STEPS=4 bash tools/gpu.sh env r4j_2048 "PFR_LANES=2" "PFR_LANES=1" "PFR_LANES=2 PFR_LEAF_SIZE=96" "PFR_LANES=1 PFR_LEAF_SIZE=96" "PFR_LANES=2" > $O/w2048.txt 2>&1 || exit $?
FREQS=1024 STEPS=5 bash tools/gpu.sh env r4j_1024 "PFR_LANES=2" "PFR_LANES=1" "PFR_LANES=2 PFR_LEAF_SIZE=96" "PFR_LANES=1 PFR_LEAF_SIZE=96" "PFR_LANES=2" > $O/w1024.txt 2>&1 || exit $?
FREQS=512 STEPS=6 bash tools/gpu.sh env r4j_512 "PFR_LANES=1" "PFR_LANES=2" "PFR_LANES=1 PFR_LEAF_SIZE=300" "PFR_LANES=1" > $O/w512.txt 2>&1 || exit $?
