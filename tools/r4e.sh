set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
O=gpurun_out/r4e
mkdir -p $O
ok() { case $1 in 0|1) return 0;; *) echo "step ended with $1: stopping"; exit "$1";; esac; }
bash tools/gpu.sh trace r4e_t2048 2048 > $O/t2048.txt 2>&1 || exit $?
python3 tools/level_times.py gpurun_out/r4e_t2048/run_kernel_trace.csv --solves > $O/t2048_solves.txt 2>&1
bash tools/gpu.sh trace r4e_t2048c2 2048 PFR_US2_CFG=2 > $O/t2048c2.txt 2>&1 || exit $?
python3 tools/level_times.py gpurun_out/r4e_t2048c2/run_kernel_trace.csv --solves > $O/t2048c2_solves.txt 2>&1
bash tools/gpu.sh traffic r4e_traffic > $O/traffic.txt 2>&1 || exit $?
PFR_US2_CFG=2 bash tools/gpu.sh traffic r4e_traffic_c2 > $O/traffic_c2.txt 2>&1 || exit $?
rm -rf gpurun_out/r4e_traffic/fetch gpurun_out/r4e_traffic/write gpurun_out/r4e_traffic_c2/fetch gpurun_out/r4e_traffic_c2/write
bash tools/gpu.sh tests r4e_tests > $O/tests.txt 2>&1; ok $?
