set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
O=gpurun_out/r4aa
mkdir -p $O
ok() { case $1 in 0|1) return 0;; *) echo "step ended with $1: stopping"; exit "$1";; esac; }
PFR_TEST_REPORT=$O/rep.jsonl timeout -k 10 400 python3 -u -m pytest tests/test_gpu_flow.py -k prefix -v --timeout 300 --timeout-method thread > $O/tests.log 2>&1; rc=$?; tail -3 $O/tests.log; ok $rc
[ $rc -eq 0 ] || exit 1
bash tools/gpu.sh trace r4aa_t2048 2048 PFR_OFF_PU=3 PFR_OFF_PU_WAVES=1000000000 > $O/t2048.txt 2>&1 || exit $?
bash tools/gpu.sh trace r4aa_t512 512 PFR_OFF_PU=3 PFR_OFF_PU_WAVES=1000000000 > $O/t512.txt 2>&1 || exit $?
rm -f gpurun_out/r4aa_t*/run_kernel_trace.csv
FREQS=4096 STEPS=4 bash tools/gpu.sh env r4aa_4096 "PFR_OFF_PU_WAVES=0" "PFR_OFF_PU=3 PFR_OFF_PU_WAVES=8000" "PFR_OFF_PU=3 PFR_OFF_PU_WAVES=1000000000" "PFR_OFF_PU_WAVES=0" "PFR_OFF_PU=3 PFR_OFF_PU_WAVES=8000" > $O/ab4096.txt 2>&1 || exit $?
FREQS=512 STEPS=8 bash tools/gpu.sh env r4aa_512 "PFR_OFF_PU_WAVES=0" "PFR_OFF_PU=3 PFR_OFF_PU_WAVES=8000" "PFR_OFF_PU=3 PFR_OFF_PU_WAVES=1000000000" "PFR_OFF_PU_WAVES=0" "PFR_OFF_PU=3 PFR_OFF_PU_WAVES=8000" > $O/ab512.txt 2>&1 || exit $?
