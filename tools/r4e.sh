set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
O=gpurun_out/r4e
mkdir -p $O
ok() { case $1 in 0|1) return 0;; *) echo "step ended with $1: stopping"; exit "$1";; esac; }
PFR_TEST_REPORT=$O/rl_report.jsonl timeout -k 10 400 python3 -u -m pytest tests/test_gpu_flow.py -k right_looking -v --timeout 300 --timeout-method thread > $O/rl_test.log 2>&1; ok $?
tail -3 $O/rl_test.log
FREQS=2048 STEPS=3 bash tools/gpu.sh env r4e_rl2048 "PFR_OFF_RL=0" "PFR_OFF_RL=16" "PFR_OFF_RL=24" "PFR_OFF_RL=32" "PFR_OFF_RL=0" "PFR_OFF_RL=32" > $O/rl2048.txt 2>&1 || exit $?
FREQS=512 STEPS=6 bash tools/gpu.sh env r4e_rl512 "PFR_OFF_RL=0" "PFR_OFF_RL=16" "PFR_OFF_RL=24" "PFR_OFF_RL=32" "PFR_OFF_RL=0" "PFR_OFF_RL=32" > $O/rl512.txt 2>&1 || exit $?
bash tools/gpu.sh trace r4e_t2048 2048 > $O/t2048.txt 2>&1 || exit $?
python3 tools/level_times.py gpurun_out/r4e_t2048/run_kernel_trace.csv --solves > $O/t2048_solves.txt 2>&1
bash tools/gpu.sh trace r4e_t2048rl 2048 PFR_OFF_RL=32 > $O/t2048rl.txt 2>&1 || exit $?
bash tools/gpu.sh trace r4e_t512rl 512 PFR_OFF_RL=32 > $O/t512rl.txt 2>&1 || exit $?
bash tools/gpu.sh trace r4e_t512 512 > $O/t512.txt 2>&1 || exit $?
bash tools/gpu.sh trace r4e_t2048c2 2048 PFR_US2_CFG=2 > $O/t2048c2.txt 2>&1 || exit $?
python3 tools/level_times.py gpurun_out/r4e_t2048c2/run_kernel_trace.csv --solves > $O/t2048c2_solves.txt 2>&1
bash tools/gpu.sh traffic r4e_traffic > $O/traffic.txt 2>&1 || exit $?
PFR_US2_CFG=2 bash tools/gpu.sh traffic r4e_traffic_c2 > $O/traffic_c2.txt 2>&1 || exit $?
rm -rf gpurun_out/r4e_traffic/fetch gpurun_out/r4e_traffic/write gpurun_out/r4e_traffic_c2/fetch gpurun_out/r4e_traffic_c2/write
for t in gpurun_out/r4e_t*/; do rm -f $t/run_kernel_trace.csv.gz; done
