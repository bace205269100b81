# Quick GPU check after a kernel change: the C3/C2 parity tests and the symmetric-mode parity tests,
# then the default bench without the CPU baseline (steps 6, warmup 2).
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:-quick}
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_fullsize.py tests/test_gpu_parity.py tests/test_gpu_symmetric.py -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1
rc=$?; tail -3 $O/tests.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u bench.py --no-cpu-baseline --steps 6 --warmup 2 > $O/bench.json 2> $O/bench.err || exit $?
python3 -c "import json;d=json.load(open('$O/bench.json'));f=d['factor_roofline'];print(round(d['value']), round(d['ms_per_step'],2), [round(x,2) for x in f['ms']], round(d['roofline']['frac'],3))"
