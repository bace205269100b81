"""Per-level durations (ms) of every factorisation / solve kernel in the LAST sweep of a
rocprofv3 --kernel-trace CSV (lanes = 1 runs: the bench's isolated sweep comes last).

Usage: python tools/level_times.py gpurun_out/<dir>/run_kernel_trace.csv [n_levels (default: the last sweep's)] [--gaps]
(--gaps: per sweep, every idle gap above 10 us between consecutive kernels, with its neighbours)
"""
import csv
import sys


LU = ("k_factor_sym", "k_factor_sym_lds", "k_factor_sym_rl", "k_factor_level", "k_front0")   # k_front0: the fused bottom level


def main(path, L=None):
    rows = list(csv.DictReader(open(path)))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    names = [r["Kernel_Name"].split("(")[0].replace("void ", "").replace("pfr::", "").split("<")[0] for r in rows]
    # one A11 LU launch per level (the assembly may be fused into it): the level marker; the level count is
    # that of the last sweep (k_chunk_start -- k_pad_freqs before round 6 -- starts every chunk)
    pads = [i for i, n in enumerate(names) if n in ("k_chunk_start", "k_pad_freqs")]
    lus = [i for i, n in enumerate(names) if n in LU and not (n == "k_front0" and names[i - 1] == "k_front0")]
    if L is None:
        L = sum(1 for i in lus if i > pads[-1]) if pads else 17
    st = lus[-L]
    # the level's assembly launch (unfused levels) precedes its LU launch
    if st > 0 and names[st - 1] == "k_assemble_level":
        st -= 1
    end = len(rows)
    tab, lvl = {}, -1
    for i, (r, n) in enumerate(zip(rows[st:end], names[st:end])):
        if n in LU or (n == "k_assemble_level" and (st + i + 1 >= end or names[st + i + 1] in LU)):
            if not (n in LU and i > 0 and names[st + i - 1] in ("k_assemble_level", "k_front0")):
                lvl += 1
        d = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6
        t = tab.setdefault(n, {})
        key = lvl if n.startswith(("k_assemble", "k_factor", "k_offdiag", "k_schur", "k_front0")) else "x"
        t[key] = t.get(key, 0.0) + d
    print("%-20s %7s " % ("kernel", "total") + " ".join("%5d" % l for l in range(L)))
    for n, t in sorted(tab.items(), key=lambda kv: -sum(kv[1].values())):
        tot = sum(t.values())
        if tot < 0.05:
            continue
        per = " ".join("%5.2f" % t.get(l, 0.0) for l in range(L)) if "x" not in t else ""
        print("%-20s %7.2f %s" % (n[:20], tot, per))
    # whole-sweep view.  A sweep = the native kernels from its k_chunk_start to its last pfr kernel (k_*); the
    # TURNAROUND before sweep k = the GPU's idle time between the end of sweep k-1's last native kernel and
    # the start of sweep k's k_chunk_start -- the host's step-to-step work (the result copy, Python, autograd,
    # the next step's buffer fills and copies); the torch / copy kernels run in that interval count as busy,
    # not idle.  (Round 5's "idle before" was measured from the previous sweep's LAST kernel of any kind,
    # which put the turnaround inside the span.)
    pads = [i for i, n in enumerate(names) if n in ("k_chunk_start", "k_pad_freqs")]
    native = [i for i, n in enumerate(names) if n.startswith("k_")]
    spans = []
    for a, b in zip(pads, pads[1:] + [len(rows)]):
        last = max(i for i in native if a <= i < b)
        t0 = int(rows[a]["Start_Timestamp"])
        t1 = int(rows[last]["End_Timestamp"])
        busy = sum(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for r in rows[a:last + 1])
        spans.append((t0, t1, busy, last + 1 - a, a, last))
    turn = []
    for k, (t0, t1, busy, nk, a, last) in enumerate(spans):
        idle = float("nan")
        if k:
            p_end, p_last = spans[k - 1][1], spans[k - 1][5]
            between = rows[p_last + 1:a]
            other = sum(min(int(r["End_Timestamp"]), t0) - max(int(r["Start_Timestamp"]), p_end) for r in between
                        if int(r["End_Timestamp"]) > p_end and int(r["Start_Timestamp"]) < t0)
            idle = (t0 - p_end - other) / 1e6
            turn.append(((t0 - p_end) / 1e6, idle))
        print("sweep %2d: span %7.3f ms  busy %7.3f ms  kernels %4d  turnaround before: %7.3f ms (GPU idle %7.3f ms)"
              % (k, (t1 - t0) / 1e6, busy / 1e6, nk, (t0 - spans[k - 1][1]) / 1e6 if k else float("nan"), idle))
        if GAPS:
            b = pads[k + 1] if k + 1 < len(pads) else len(rows)
            for i in range(a + 1, b):
                g = (int(rows[i]["Start_Timestamp"]) - int(rows[i - 1]["End_Timestamp"])) / 1e3
                if g > 10:
                    print("    gap %8.1f us  %-24s -> %s" % (g, names[i - 1][:24], names[i][:24]))
    if turn:
        steady = turn[1:] or turn
        print("turnaround between consecutive sweeps (steady, sweeps 2..): mean %.3f ms, GPU idle mean %.3f ms, max %.3f ms"
              % (sum(t for t, _ in steady) / len(steady), sum(i for _, i in steady) / len(steady),
                 max(i for _, i in steady)))


GAPS = "--gaps" in sys.argv
SOLVES = "--solves" in sys.argv


def solves(path):
    """The last sweep's solve launches in order: per kernel, (duration us) -- the paired top-down pass
    runs its levels top first, so its k_usolve2_level launches map to levels L-1 .. 0."""
    rows = list(csv.DictReader(open(path)))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    names = [r["Kernel_Name"].split("(")[0].replace("void ", "").replace("pfr::", "") for r in rows]
    pads = [i for i, n in enumerate(names) if n.startswith(("k_chunk_start", "k_pad_freqs"))]
    a = pads[-1] if pads else 0
    seq = {}
    for r, n in zip(rows[a:], names[a:]):
        if "solve" in n or n.startswith(("k_fn_", "k_residual", "k_dirichlet")):
            key = n.split("(")[0]
            seq.setdefault(key, []).append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
    for k, v in seq.items():
        print("%-44s n %3d  total %7.1f us" % (k[:44], len(v), sum(v)))
        print("    " + " ".join("%.0f" % x for x in v))


if __name__ == "__main__":
    args = [a for a in sys.argv[1:] if a not in ("--gaps", "--solves")]
    if SOLVES:
        solves(args[0])
    else:
        main(args[0], int(args[1]) if len(args) > 1 else None)
