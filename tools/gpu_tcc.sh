# L2 hit/miss per kernel (rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum), one lanes=1 bench step at 2,048 frequencies
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:-tcc}
mkdir -p $O
PFR_LANES=1 timeout -s KILL 120 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum --kernel-trace --output-format csv -d $O -o run -- python3 bench.py --steps 1 --warmup 0 --freqs 2048 --no-cpu-baseline > $O/bench.json 2> $O/err.txt && echo DONE
