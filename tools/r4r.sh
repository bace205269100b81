set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
O=gpurun_out/r4r
mkdir -p $O
ok() { case $1 in 0|1) return 0;; *) echo "step ended with $1: stopping"; exit "$1";; esac; }
PFR_TEST_REPORT=$O/rep.jsonl timeout -k 10 400 python3 -u -m pytest tests/test_gpu_flow.py -k tiny -v --timeout 300 --timeout-method thread > $O/tests.log 2>&1; ok $?
tail -3 $O/tests.log
FREQS=2048 STEPS=4 bash tools/gpu.sh env r4r_2048 "PFR_US2_TINY=8" "PFR_US2_TINY=16" "PFR_US2_TINY=24" "PFR_US2_TINY=40" "PFR_US2_TINY=8" "PFR_US2_TINY=16" > $O/ab2048.txt 2>&1 || exit $?
FREQS=512 STEPS=8 bash tools/gpu.sh env r4r_512 "PFR_US2_TINY=8" "PFR_US2_TINY=16" "PFR_US2_TINY=24" "PFR_US2_TINY=40" "PFR_US2_TINY=8" "PFR_US2_TINY=16" > $O/ab512.txt 2>&1 || exit $?
bash tools/gpu.sh trace r4r_t2048 2048 PFR_US2_TINY=24 > $O/t2048.txt 2>&1 || exit $?
python3 tools/level_times.py gpurun_out/r4r_t2048/run_kernel_trace.csv --solves > $O/t2048_solves.txt 2>&1
rm -f gpurun_out/r4r_t2048/run_kernel_trace.csv
