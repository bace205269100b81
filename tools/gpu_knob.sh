# A/B of a runtime knob: the parity / check tests with KNOB set, then kernel-class times and the default
# two-lane bench with and without it.   bash tools/gpu_knob.sh OUT "KNOB=V [KNOB2=V2]"
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:-knob}
K="$2"
mkdir -p $O
env $K timeout -k 10 600 python -u -m pytest tests/test_gpu_fullsize.py tests/test_gpu_parity.py tests/test_gpu_symmetric.py tests/test_gpu_check.py -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1
rc=$?; tail -3 $O/tests.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 600 bash tools/exp_env.sh "PFR_LANES=1" "PFR_LANES=1 $K" || exit $?
for cfg in "" "$K" "" "$K"; do
  env $cfg timeout -k 10 300 python -u bench.py --no-cpu-baseline --steps 8 --warmup 2 > $O/bench.json 2> $O/bench.err || exit $?
  python3 -c "import json;d=json.load(open('$O/bench.json'));print('$cfg |', round(d['value']), round(d['ms_per_step'],2))"
done
