# One SQ-counter pass over a bench step (lanes = 1): wave cycles split into parked / issue-stalled / active
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp PFR_LANES=1
O=gpurun_out/${1:-sq}
mkdir -p $O
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_VMEM SQ_WAVES SQ_BUSY_CYCLES --kernel-trace --output-format csv -d $O/sq -o run -- python3 bench.py --steps 1 --warmup 0 --freqs 2048 --no-cpu-baseline > $O/sq.json 2> $O/sq.err
rc=$?
tail -2 $O/sq.err
exit $rc
