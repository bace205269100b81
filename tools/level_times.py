"""Per-level durations (ms) of every factorisation / solve kernel in the LAST sweep of a
rocprofv3 --kernel-trace CSV (lanes = 1 runs: the bench's isolated sweep comes last).

Usage: python tools/level_times.py gpurun_out/<dir>/run_kernel_trace.csv [n_levels=17]
"""
import csv
import sys


def main(path, L=17):
    rows = list(csv.DictReader(open(path)))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    names = [r["Kernel_Name"].split("(")[0].replace("void ", "").replace("pfr::", "").split("<")[0] for r in rows]
    asm = [i for i, n in enumerate(names) if n == "k_assemble_level"]
    st = asm[-L]
    end = len(rows)
    tab, lvl = {}, -1
    for r, n in zip(rows[st:end], names[st:end]):
        if n == "k_assemble_level":
            lvl += 1
        d = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6
        t = tab.setdefault(n, {})
        key = lvl if n.startswith(("k_assemble", "k_factor", "k_offdiag", "k_schur")) else "x"
        t[key] = t.get(key, 0.0) + d
    print("%-20s %7s " % ("kernel", "total") + " ".join("%5d" % l for l in range(L)))
    for n, t in sorted(tab.items(), key=lambda kv: -sum(kv[1].values())):
        tot = sum(t.values())
        if tot < 0.05:
            continue
        per = " ".join("%5.2f" % t.get(l, 0.0) for l in range(L)) if "x" not in t else ""
        print("%-20s %7.2f %s" % (n[:20], tot, per))


if __name__ == "__main__":
    main(sys.argv[1], int(sys.argv[2]) if len(sys.argv) > 2 else 17)
