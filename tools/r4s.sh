set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
O=gpurun_out/r4s
mkdir -p $O
FREQS=4096 STEPS=4 bash tools/gpu.sh env r4s_4096 "PFR_FAC_LDS_WG=160" "PFR_FAC_LDS_WG=300" "PFR_MAX_NS=64" "PFR_MAX_NS=64 PFR_FAC_LDS_WG=300" "PFR_FAC_LDS_WG=160" "PFR_MAX_NS=48 PFR_FAC_LDS_WG=300" > $O/ab4096.txt 2>&1 || exit $?
bash tools/gpu.sh trace r4s_t2048 2048 PFR_MAX_NS=64 PFR_FAC_LDS_WG=300 > $O/t2048.txt 2>&1 || exit $?
rm -f gpurun_out/r4s_t2048/run_kernel_trace.csv
