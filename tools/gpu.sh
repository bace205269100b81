# One launcher for every GPU-box job (run through gpurun from the repository root):
#
#   bash tools/gpu.sh tests   OUT [pytest args]       GPU tests, per-test error report (OUT/test_report.jsonl)
#   bash tools/gpu.sh quick   OUT                     C3/C2 + symmetric parity tests, then the bench (no CPU leg)
#   bash tools/gpu.sh bench   OUT [bench args]        bench.py
#   bash tools/gpu.sh stats   OUT [bench args]        rocprofv3 --kernel-trace --stats of the bench, one lane,
#                                                     2,048-frequency chunks (isolated launches)
#   bash tools/gpu.sh traffic OUT                     FETCH_SIZE / WRITE_SIZE passes (separate runs) of one
#                                                     lanes=1 2,048-frequency step -> OUT/pmc_traffic.json
#   bash tools/gpu.sh pmc     OUT COUNTER...          one --pmc pass over the same step (counter limits per
#                                                     block: see MI355X_MICROARCH.md)
#   bash tools/gpu.sh trace   OUT F [ENV=V ...]       kernel trace of one lanes=1 step of F frequencies in one
#                                                     chunk + per-level times (tools/level_times.py)
#   bash tools/gpu.sh env     OUT "ENV=V ..." ...     kernel-class times of one isolated chunk per setting
#                                                     (FREQS frequencies, STEPS timed steps)
#   bash tools/gpu.sh strong  OUT                     1-GPU strong-scaling proxy (tools/strong_proxy.py)
#   bash tools/gpu.sh round   R                       round measurement: tests, traffic (-> profiles/R),
#                                                     bench, stats, C5, strong proxy, 6-step 512 trace
#
# Every GPU step runs under its own time limit; the script stops at the first failure and never
# starts another GPU step after a timeout / abort / fault (exit 124, 134, 137, 139).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
CMD=$1
O=gpurun_out/${2:-$1}
shift 2 2>/dev/null || shift $#
mkdir -p "$O"
STEP="python3 bench.py --steps 1 --warmup 0 --freqs 2048 --no-cpu-baseline"

stop() { case $1 in 0) ;; 124|134|137|139) echo "step ended with $1: stopping"; exit "$1";; *) exit "$1";; esac; }

tests() {
  rm -f "$O/test_report.jsonl"
  PFR_TEST_REPORT=$O/test_report.jsonl timeout -k 10 1100 python3 -u -m pytest tests -m gpu -v --timeout 300 \
    --timeout-method thread "$@" > "$O/gpu_tests.log" 2>&1
  local rc=$?; tail -4 "$O/gpu_tests.log"; return $rc
}
bench() { timeout -k 10 400 python3 -u bench.py "$@" > "$O/bench.json" 2> "$O/bench.err"; local rc=$?; cat "$O/bench.json"; tail -3 "$O/bench.err"; return $rc; }
stats() {
  PFR_LANES=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/stats" -o run -- \
    python3 bench.py --no-cpu-baseline --no-strong-proxy --chunk 2048 "$@" > "$O/bench_lanes1_chunk2048.json" 2> "$O/stats.err"
}
traffic() {
  PFR_LANES=1 timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d "$O/fetch" -o run -- \
    $STEP > "$O/fetch.json" 2> "$O/fetch.err" || return $?
  PFR_LANES=1 timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d "$O/write" -o run -- \
    $STEP > "$O/write.json" 2> "$O/write.err" || return $?
  python3 tools/pmc_summary.py "$O/fetch" "$O/write" --last-sweep --freqs 2048 --json "$O/pmc_traffic.json" \
    --note "rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE (separate passes) --kernel-trace of: PFR_LANES=1 $STEP; last sweep (timed step + isolated sweep)" \
    > "$O/pmc_summary.txt"
}
pmc() {
  PFR_LANES=1 timeout -s KILL 120 rocprofv3 --pmc "$@" --kernel-trace --output-format csv -d "$O/pmc" -o run -- \
    $STEP > "$O/pmc.json" 2> "$O/pmc.err" || { tail -3 "$O/pmc.err"; return 1; }
}
trace() {
  local F=${1:-2048}; shift
  env PFR_LANES=1 "$@" timeout -k 10 240 rocprofv3 --kernel-trace --output-format csv -d "$O" -o run -- \
    python3 bench.py --steps "${STEPS:-1}" --warmup 0 --freqs "$F" --chunk "$F" --no-cpu-baseline > "$O/b.json" 2> "$O/err" || return $?
  python3 tools/level_times.py "$O/run_kernel_trace.csv"
}
envs() {
  local i=0 cfg
  for cfg in "$@"; do
    i=$((i + 1))
    env $cfg timeout -k 10 200 python3 -u bench.py --no-cpu-baseline --no-strong-proxy --steps "${STEPS:-3}" --freqs "${FREQS:-2048}" \
      > "$O/e$i.json" 2> "$O/e$i.err" || { tail -5 "$O/e$i.err"; return 1; }
    python3 -c "import json;d=json.load(open('$O/e$i.json'));f=d['factor_roofline'];p=d['phase_ms'];print('$cfg |', round(d['value']), [round(x,2) for x in f['ms']], {k:round(v,2) for k,v in p.items() if k!='note'})"
  done
}
strong() { timeout -k 10 400 python3 -u tools/strong_proxy.py --out "$O/strong_proxy.json" > "$O/strong.log" 2>&1; local rc=$?; tail -12 "$O/strong.log"; return $rc; }

case $CMD in
  tests) tests "$@" ;;
  quick)
    timeout -k 10 600 python3 -u -m pytest tests/test_gpu_fullsize.py tests/test_gpu_parity.py tests/test_gpu_symmetric.py \
      -x -q --timeout 300 --timeout-method thread > "$O/tests.log" 2>&1
    rc=$?; tail -3 "$O/tests.log"; stop $rc
    bench --no-cpu-baseline --no-strong-proxy --steps 6 --warmup 2 ;;
  bench) bench "$@" ;;
  stats) stats "$@" ;;
  traffic) traffic ;;
  pmc) pmc "$@" ;;
  trace) trace "$@" ;;
  env) envs "$@" ;;
  strong) strong ;;
  round)
    R=${O#gpurun_out/}
    tests; rc=$?; stop $rc
    traffic; stop $?
    mkdir -p "profiles/$R" && cp "$O/pmc_traffic.json" "profiles/$R/pmc_traffic.json"
    bench; stop $?
    stats; stop $?
    timeout -k 10 600 python3 -u tools/c5_lbfgs.py > "$O/c5.json" 2> "$O/c5.err"; stop $?
    cat "$O/c5.json"
    strong; stop $?
    mkdir -p "$O/tr512" && (O=$O/tr512; STEPS=6 trace 512) > "$O/tr512/levels.txt" 2>&1; stop $?
    echo DONE ;;
  *) echo "unknown command $CMD"; exit 2 ;;
esac
