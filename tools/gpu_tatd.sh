# Texture-path stall counters per dispatch, one lanes=1 bench step at 2,048 frequencies (four passes):
#   a: TA busy, TA address stalled by the cache;  b: TA data stalled by the cache, TA stalled by TD;
#   c: TD busy, TD waiting on the cache;  d: L1 pending / tag-conflict / return stalls, L1->L2 reads
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp PFR_LANES=1
O=gpurun_out/${1:-tatd}
mkdir -p $O
run() { timeout -s KILL 120 rocprofv3 --pmc "$@" --kernel-trace --output-format csv -d $O/p$N -o run -- python3 bench.py --steps 1 --warmup 0 --freqs 2048 --no-cpu-baseline > $O/p$N.json 2> $O/p$N.err || { tail -3 $O/p$N.err; exit 1; }; }
N=a run TA_TA_BUSY_sum TA_ADDR_STALLED_BY_TC_CYCLES_sum GRBM_GUI_ACTIVE
N=b run TA_DATA_STALLED_BY_TC_CYCLES_sum TA_ADDR_STALLED_BY_TD_CYCLES_sum GRBM_GUI_ACTIVE
N=c run TD_TD_BUSY_sum TD_TC_STALL_sum GRBM_GUI_ACTIVE
N=d run TCP_PENDING_STALL_CYCLES_sum TCP_READ_TAGCONFLICT_STALL_CYCLES_sum TCP_TCR_TCP_STALL_CYCLES_sum TCP_TCC_READ_REQ_sum GRBM_GUI_ACTIVE
echo DONE
