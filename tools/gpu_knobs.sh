# Kernel-class times (one lane, one 2,048-frequency chunk) and the default bench for several knob
# settings, after the parity tests under the first:  bash tools/gpu_knobs.sh OUT "K=V ..." "K=V ..."
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:-knobs}
shift
mkdir -p $O
env $1 timeout -k 10 600 python -u -m pytest tests/test_gpu_fullsize.py tests/test_gpu_parity.py tests/test_gpu_symmetric.py -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1
rc=$?; tail -3 $O/tests.log
[ $rc -ne 0 ] && exit $rc
cfgs=("PFR_LANES=1")
for k in "$@"; do cfgs+=("PFR_LANES=1 $k"); done
timeout -k 10 900 bash tools/exp_env.sh "${cfgs[@]}" || exit $?
for cfg in "" "$@"; do
  env $cfg timeout -k 10 300 python -u bench.py --no-cpu-baseline --steps 8 --warmup 2 > $O/bench.json 2> $O/bench.err || exit $?
  python3 -c "import json;d=json.load(open('$O/bench.json'));print('$cfg |', round(d['value']), round(d['ms_per_step'],2))"
done
