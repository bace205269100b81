# Memory-pipeline counters per kernel, one lanes=1 bench step at 2,048 frequencies (three passes):
#   A: L1->L2 read requests and their summed latency, L1 accesses, TA busy;  B: L2 hits / misses,
#   L2 busy, TD busy;  C: EA read-request queue level, L2 tag stalls
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp PFR_LANES=1
O=gpurun_out/${1:-mem}
mkdir -p $O
run() { timeout -s KILL 120 rocprofv3 --pmc "$@" --kernel-trace --output-format csv -d $O/p$N -o run -- python3 bench.py --steps 1 --warmup 0 --freqs 2048 --no-cpu-baseline > $O/p$N.json 2> $O/p$N.err || { tail -3 $O/p$N.err; exit 1; }; }
N=a run TCP_TCC_READ_REQ_sum TCP_TCC_READ_REQ_LATENCY_sum TCP_TOTAL_CACHE_ACCESSES_sum TA_BUSY_avr GRBM_GUI_ACTIVE
N=b run TCC_HIT_sum TCC_MISS_sum TCC_BUSY_avr TD_TD_BUSY_sum GRBM_GUI_ACTIVE
N=c run TCC_EA0_RDREQ_LEVEL_sum TCC_TAG_STALL_sum GRBM_GUI_ACTIVE
echo DONE
