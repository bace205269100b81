# Round-2 GPU check: all GPU tests (no -x; per-test report), then the default bench.
# Stops before the bench if the tests ended by a timeout / abort / signal (124, 134, 137, 139).
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:-r2}
mkdir -p $O
rm -f $O/test_report.jsonl
PFR_TEST_REPORT=$O/test_report.jsonl timeout -k 10 1000 python -u -m pytest tests -m gpu -v --timeout 300 \
  --timeout-method thread ${PYTEST_K:+-k "$PYTEST_K"} > $O/gpu_tests.log 2>&1
rc=$?
tail -12 $O/gpu_tests.log
case $rc in 124|134|137|139) echo "tests ended with $rc: stopping"; exit $rc;; esac
[ -n "$NO_BENCH" ] && exit $rc
timeout -k 10 400 python -u bench.py ${BENCH_ARGS:-} > $O/bench.json 2> $O/bench.err
brc=$?
cat $O/bench.json
tail -3 $O/bench.err
[ $rc -ne 0 ] && exit $rc
exit $brc
