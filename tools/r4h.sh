set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
O=gpurun_out/r4h
mkdir -p $O
ok() { case $1 in 0|1) return 0;; *) echo "step ended with $1: stopping"; exit "$1";; esac; }
PFR_TEST_REPORT=$O/rep.jsonl timeout -k 10 600 python3 -u -m pytest tests/test_gpu_flow.py tests/test_gpu_c5.py -k "right_looking or c5" -v --timeout 400 --timeout-method thread > $O/tests.log 2>&1; ok $?
tail -4 $O/tests.log
FREQS=2048 STEPS=3 bash tools/gpu.sh env r4h_rl2048 "PFR_OFF_RL=0" "PFR_OFF_RL=116" "PFR_OFF_RL=124" "PFR_OFF_RL=0" "PFR_OFF_RL=116" > $O/rl2048.txt 2>&1 || exit $?
FREQS=512 STEPS=6 bash tools/gpu.sh env r4h_rl512 "PFR_OFF_RL=0" "PFR_OFF_RL=116" "PFR_OFF_RL=124" "PFR_OFF_RL=0" "PFR_OFF_RL=116" > $O/rl512.txt 2>&1 || exit $?
bash tools/gpu.sh trace r4h_t2048 2048 PFR_OFF_RL=116 > $O/t2048rl116.txt 2>&1 || exit $?
rm -f gpurun_out/r4h_t2048/run_kernel_trace.csv
FREQS=4096 STEPS=4 bash tools/gpu.sh env r4h_lanes "PFR_LANES=2" "PFR_LANES=1" "PFR_LANES=2" "PFR_LANES=1" > $O/lanes4096.txt 2>&1 || exit $?
