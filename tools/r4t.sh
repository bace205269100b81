set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
O=gpurun_out/r4t
mkdir -p $O
FREQS=4096 STEPS=5 bash tools/gpu.sh env r4t_4096 "PFR_LANE_PRIO=0" "PFR_LANE_PRIO=1" "PFR_LANE_PRIO=0" "PFR_LANE_PRIO=1" "PFR_LANE_PRIO=1 PFR_LANES=3" > $O/ab4096.txt 2>&1 || exit $?
FREQS=2048 STEPS=5 bash tools/gpu.sh env r4t_2048 "PFR_LANE_PRIO=0" "PFR_LANE_PRIO=1" "PFR_LANE_PRIO=0" "PFR_LANE_PRIO=1" > $O/ab2048.txt 2>&1 || exit $?
FREQS=1024 STEPS=6 bash tools/gpu.sh env r4t_1024 "PFR_LANE_PRIO=0" "PFR_LANE_PRIO=1" "PFR_LANE_PRIO=0" "PFR_LANE_PRIO=1" > $O/ab1024.txt 2>&1 || exit $?
