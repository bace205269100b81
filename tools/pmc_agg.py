"""Sum rocprofv3 --pmc counters per kernel (all dispatches) and print them with ratios.

Usage: python tools/pmc_agg.py gpurun_out/<dir>/run_counter_collection.csv [kernel prefixes ...]
"""
import collections
import csv
import sys


def load(path):
    agg = collections.defaultdict(lambda: collections.defaultdict(float))
    for r in csv.DictReader(open(path)):
        n = r["Kernel_Name"].split("(")[0].replace("void ", "").replace("pfr::", "")
        agg[n][r["Counter_Name"]] += float(r["Counter_Value"])
    return agg


def main():
    agg = load(sys.argv[1])
    pref = sys.argv[2:] or ["k_"]
    for n, d in sorted(agg.items(), key=lambda kv: -sum(kv[1].values())):
        if not any(n.startswith(p) for p in pref):
            continue
        print("%-34s " % n[:34] + "  ".join("%s=%.3g" % (k.replace("_sum", ""), v) for k, v in sorted(d.items())))


if __name__ == "__main__":
    main()
