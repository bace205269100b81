set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
O=gpurun_out/r4i
mkdir -p $O
L=$PWD/plate_inverse_problem_amd/_lib
bash tools/gpu.sh trace r4i_t2048_rpl4 2048 PFR_LIB=$L/libpfr_rpl4.so > $O/t2048_rpl4.txt 2>&1 || exit $?
bash tools/gpu.sh trace r4i_t2048_rpl1 2048 PFR_LIB=$L/libpfr_rpl1.so > $O/t2048_rpl1.txt 2>&1 || exit $?
bash tools/gpu.sh trace r4i_t512_rpl4 512 PFR_LIB=$L/libpfr_rpl4.so > $O/t512_rpl4.txt 2>&1 || exit $?
bash tools/gpu.sh trace r4i_t512_rpl1 512 PFR_LIB=$L/libpfr_rpl1.so > $O/t512_rpl1.txt 2>&1 || exit $?
rm -f gpurun_out/r4i_t*/run_kernel_trace.csv
