"""Per-level SQ / TCC counters of the last 512-frequency sweep in a tools/pmc_levels.sh run:
    python tools/pmc_levels.py gpurun_out/<dir>
Per factorisation class and level: duration (us), waves, SQ_WAIT_ANY / SQ_WAVE_CYCLES, VALU busy share,
VMEM reads per wave, L2 hit rate."""
import collections
import csv
import sys

LU = ("k_factor_sym", "k_factor_sym_lds", "k_factor_level", "k_front0")


def load(path):
    d = collections.OrderedDict()
    for r in csv.DictReader(open(path)):
        k = int(r["Dispatch_Id"])
        e = d.setdefault(k, {"name": r["Kernel_Name"].split("(")[0].replace("void ", "").replace("pfr::", ""),
                             "t": (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3,
                             "start": int(r["Start_Timestamp"]), "grid": int(r["Grid_Size"]),
                             "wg": int(r["Workgroup_Size"])})
        e[r["Counter_Name"]] = float(r["Counter_Value"])
    return list(d.values())


def main(o):
    sq, tc = load(o + "/sq/run_counter_collection.csv"), load(o + "/tcc/run_counter_collection.csv")
    # the last sweep: from the last k_chunk_start / k_pad_freqs
    def last(rows):
        st = max(i for i, r in enumerate(rows) if r["name"].startswith(("k_chunk_start", "k_pad_freqs")))
        return rows[st:]
    sq, tc = last(sq), last(tc)
    lvl, out = -1, []
    for a, b in zip(sq, tc):
        base = a["name"].split("<")[0]
        if base in LU:
            lvl += 1
        if base == "k_assemble_level":
            lvl += 1 if lvl >= 0 else 1
        wc = a.get("SQ_WAVE_CYCLES", 0) or 1
        hit, miss = b.get("TCC_HIT_sum", 0), b.get("TCC_MISS_sum", 0)
        out.append((lvl, a["name"][:34], a["t"], a["grid"] // 64, a.get("SQ_WAIT_ANY", 0) / wc,
                    a.get("SQ_ACTIVE_INST_VALU", 0) / wc, a.get("SQ_INSTS_VMEM_RD", 0) / max(1, a.get("SQ_WAVES", 1)),
                    hit / max(1, hit + miss)))
    print("%-4s %-34s %8s %7s %6s %6s %9s %6s" % ("lvl", "kernel", "us", "waves", "wait", "valu", "vmem/wave", "L2hit"))
    for r in out:
        print("%-4d %-34s %8.1f %7d %6.2f %6.2f %9.1f %6.2f" % r)


if __name__ == "__main__":
    main(sys.argv[1])
