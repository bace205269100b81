# Alternated A/B of environment settings on the headline workload (bench.py, 4,096 frequencies, a fresh process each):
#   REPS=3 STEPS=10 bash tools/ab_bench.sh OUTDIR "PFR_X=1" "PFR_X=0" ...
O=gpurun_out/$1; shift
mkdir -p "$O"
for i in $(seq 1 "${REPS:-3}"); do
  k=0
  for cfg in "$@"; do
    k=$((k + 1))
    env $cfg timeout -k 10 200 python3 -u bench.py --no-cpu-baseline --no-strong-proxy --steps "${STEPS:-10}" --warmup 2 \
      > "$O/b${k}_$i.json" 2> "$O/b${k}_$i.err" || { tail -5 "$O/b${k}_$i.err"; exit 1; }
    echo "$cfg | $(python3 -c "import json;d=json.load(open('$O/b${k}_$i.json'));print(round(d['value']), round(d['ms_per_step'],2), [round(x,2) for x in d['factor_roofline']['ms']])")"
  done
done
