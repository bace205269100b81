# Address-translation and L1 latency counters per kernel, one lanes=1 bench step at 2,048 frequencies
# (two passes: UTCL1 requests / hits / misses + UTCL2 busy; TCP latency and stall cycles)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp PFR_LANES=1
O=gpurun_out/${1:-tlb}
mkdir -p $O
timeout -s KILL 120 rocprofv3 --pmc TCP_UTCL1_REQUEST_sum TCP_UTCL1_TRANSLATION_HIT_sum TCP_UTCL1_TRANSLATION_MISS_sum TCP_UTCL1_PERMISSION_MISS_sum GRBM_UTCL2_BUSY GRBM_GUI_ACTIVE --kernel-trace --output-format csv -d $O/a -o run -- python3 bench.py --steps 1 --warmup 0 --freqs 2048 --no-cpu-baseline > $O/a.json 2> $O/a.err || { tail -3 $O/a.err; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc TCP_TCP_LATENCY_sum TCP_TCC_READ_REQ_LATENCY_sum TCP_PENDING_STALL_CYCLES_sum TCP_TCR_TCP_STALL_CYCLES_sum --kernel-trace --output-format csv -d $O/b -o run -- python3 bench.py --steps 1 --warmup 0 --freqs 2048 --no-cpu-baseline > $O/b.json 2> $O/b.err || { tail -3 $O/b.err; exit 1; }
echo DONE
