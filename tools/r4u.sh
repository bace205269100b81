set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
O=gpurun_out/r4u
mkdir -p $O
ok() { case $1 in 0|1) return 0;; *) echo "step ended with $1: stopping"; exit "$1";; esac; }
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_debug_solution.py -v --timeout 200 --timeout-method thread > $O/dbg.log 2>&1; ok $?
tail -3 $O/dbg.log
L=$PWD/plate_inverse_problem_amd/_lib
for v in g2 g2r1; do
  bash tools/gpu.sh trace r4u_t2048_$v 2048 PFR_LIB=$L/libpfr_$v.so > $O/t2048_$v.txt 2>&1 || exit $?
  bash tools/gpu.sh trace r4u_t512_$v 512 PFR_LIB=$L/libpfr_$v.so > $O/t512_$v.txt 2>&1 || exit $?
done
rm -f gpurun_out/r4u_t*/run_kernel_trace.csv
