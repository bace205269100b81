"""Per-level durations of chosen kernels from tools/gpu.sh trace runs (last sweep).

Usage: python tools/trace_levels.py gpurun_out/trace/t1 [t2 ...] [--kernels schur,offdiag]
"""
import csv
import sys


def load(d):
    rows = list(csv.DictReader(open(d + "/run_kernel_trace.csv")))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    names = [r["Kernel_Name"].split("(")[0].replace("void ", "").replace("pfr::", "") for r in rows]
    st = max(i for i, n in enumerate(names) if "k_combine" in n)
    out = {}
    lvl = -1
    for r, n in zip(rows[st:], names[st:]):
        if "assemble" in n:
            lvl += 1
        key = n.split("<")[0]
        out.setdefault(key, []).append((lvl, (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6))
    return out


def main():
    args = [a for a in sys.argv[1:] if not a.startswith("--")]
    ks = ["k_schur", "k_offdiag_level", "k_factor_level", "k_assemble_level", "k_usolve_level", "k_lsolve_level"]
    for a in sys.argv[1:]:
        if a.startswith("--kernels="):
            ks = a.split("=", 1)[1].split(",")
    data = [(open(d + "/cfg").read().strip(), load(d)) for d in args]
    for k in ks:
        print("==", k)
        for cfg, dd in data:
            vals = []
            for key, lst in dd.items():
                if key.startswith(k):
                    vals = lst
            first = vals[:15]
            print("%-34s tot %7.2f  " % (cfg[:34], sum(v for _, v in first)) + " ".join("%5.2f" % v for _, v in first))


if __name__ == "__main__":
    main()
