set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
O=gpurun_out/r4o
mkdir -p $O
bash tools/gpu.sh trace r4o_t512 512 PFR_OFF_SWZ_MIN=1000000000 > $O/t512_noswz.txt 2>&1 || exit $?
bash tools/gpu.sh trace r4o_t512b 512 > $O/t512.txt 2>&1 || exit $?
bash tools/gpu.sh trace r4o_t2048 2048 PFR_OFF_SWZ_MIN=1000000000 > $O/t2048_noswz.txt 2>&1 || exit $?
rm -f gpurun_out/r4o_t*/run_kernel_trace.csv
FREQS=512 STEPS=8 bash tools/gpu.sh env r4o_512 "PFR_OFF_SWZ_MIN=0" "PFR_OFF_SWZ_MIN=1000000000" "PFR_OFF_SWZ_MIN=0" "PFR_OFF_SWZ_MIN=1000000000" > $O/ab512.txt 2>&1 || exit $?
