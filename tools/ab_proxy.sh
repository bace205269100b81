# Alternated A/B of environment settings on C4's rank block (tools/strong_proxy.py --one N, a fresh process each):
#   REPS=3 N=512 bash tools/ab_proxy.sh OUTDIR "PFR_X=1" "PFR_X=0" ...
O=gpurun_out/$1; shift
mkdir -p "$O"
for i in $(seq 1 "${REPS:-3}"); do
  k=0
  for cfg in "$@"; do
    k=$((k + 1))
    env $cfg timeout -k 10 120 python3 tools/strong_proxy.py --one "${N:-512}" 0 --steps "${STEPS:-20}" --warmup 3 \
      > "$O/p${k}_$i.json" 2>/dev/null || exit 1
    echo "$cfg | $(python3 -c "import json;d=json.load(open('$O/p${k}_$i.json'));print(round(d['freq_solves_per_s']), round(d['ms_per_step'],3), d['lanes'])")"
  done
done
