"""Per-level factorisation kernel table from rocprofv3 FETCH_SIZE / WRITE_SIZE passes.

Usage: python tools/level_table.py PROFDIR   (PROFDIR holds fetch/ and write/ as written by
tools/gpu.sh traffic / stats).  Prints, for the last sweep (after the last k_combine), every
factorisation launch with its level, duration, HBM read/write (FETCH_SIZE x2, gfx950) and
rate.
"""
import csv
import sys


def load(d):
    return list(csv.DictReader(open(d + "/run_counter_collection.csv")))


def main(d):
    f, w = load(d + "/fetch"), load(d + "/write")
    wd = {int(r["Dispatch_Id"]): float(r["Counter_Value"]) * 1024 for r in w}
    names = [r["Kernel_Name"].split("(")[0].replace("void ", "").replace("pfr::", "") for r in f]
    st = max(i for i, n in enumerate(names) if "k_combine" in n)
    lvl = -1
    tot = {}
    print("%-24s %5s %8s %8s %8s %7s" % ("kernel", "lvl", "ms", "rdGB", "wrGB", "TB/s"))
    for r, n in zip(f[st:], names[st:]):
        if "assemble" in n:
            lvl += 1
        dt = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6
        rd = 2 * float(r["Counter_Value"]) * 1024
        wr = wd.get(int(r["Dispatch_Id"]), 0)
        t = tot.setdefault(n, [0, 0, 0])
        t[0] += dt; t[1] += rd; t[2] += wr
        if ALL or any(k in n for k in ["schur", "offdiag", "factor", "assemble"]):
            print("%-24s %5d %8.3f %8.2f %8.2f %7.2f" % (n[:24], lvl, dt, rd / 1e9, wr / 1e9, (rd + wr) / dt / 1e9))
    print()
    for n, (dt, rd, wr) in sorted(tot.items(), key=lambda kv: -kv[1][0]):
        print("%-40s %8.2f ms %8.2f GB rd %8.2f GB wr" % (n[:40], dt, rd / 1e9, wr / 1e9))


ALL = "--all" in sys.argv

if __name__ == "__main__":
    main(sys.argv[1])
