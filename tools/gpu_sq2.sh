# Two SQ-counter passes over one lanes=1 bench step at 2,048 frequencies:
#   A: wave cycles parked / issue-stalled / active, VALU / VMEM activity
#   B: instruction counts (VALU, LDS, VMEM reads), LDS issue stalls and bank conflicts
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp PFR_LANES=1
O=gpurun_out/${1:-sq}
mkdir -p $O
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_VMEM SQ_WAVES SQ_BUSY_CYCLES --kernel-trace --output-format csv -d $O/a -o run -- python3 bench.py --steps 1 --warmup 0 --freqs 2048 --no-cpu-baseline > $O/a.json 2> $O/a.err || { tail -3 $O/a.err; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_VMEM_RD SQ_ACTIVE_INST_LDS SQ_INSTS_SALU --kernel-trace --output-format csv -d $O/b -o run -- python3 bench.py --steps 1 --warmup 0 --freqs 2048 --no-cpu-baseline > $O/b.json 2> $O/b.err || { tail -3 $O/b.err; exit 1; }
echo DONE
