mkdir -p gpurun_out/r6u
for i in 1 2 3; do
  for lf in 256 512; do
    PFR_LANE_FREQS=$lf timeout -k 10 120 python3 tools/strong_proxy.py --one 512 0 --steps 20 --warmup 3 > gpurun_out/r6u/p_${lf}_$i.json 2>/dev/null || exit 1
    echo "$lf $(cat gpurun_out/r6u/p_${lf}_$i.json)"
  done
done
