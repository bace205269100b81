# Per-dispatch SQ / TCC counters of one 512-frequency sweep on one lane (each pass its own run):
#   bash tools/pmc_levels.sh OUTDIR
O=gpurun_out/$1
mkdir -p "$O"
STEP="python3 bench.py --steps 1 --warmup 0 --freqs 512 --chunk 512 --no-cpu-baseline --no-strong-proxy"
PFR_LANES=1 timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VMEM_RD SQ_BUSY_CYCLES SQ_WAVES SQ_INSTS_VALU \
  --kernel-trace --output-format csv -d "$O/sq" -o run -- $STEP > "$O/sq.json" 2> "$O/sq.err" || { tail -3 "$O/sq.err"; exit 1; }
PFR_LANES=1 timeout -s KILL 120 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum TCP_TCC_READ_REQ_sum \
  --kernel-trace --output-format csv -d "$O/tcc" -o run -- $STEP > "$O/tcc.json" 2> "$O/tcc.err" || { tail -3 "$O/tcc.err"; exit 1; }
echo done
