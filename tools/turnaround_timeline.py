"""Host marks (tools/host_turnaround.py with HT_DUMP) lined up with the rocprofv3 kernel trace of the same run:
per step, from the end of the last native kernel of the previous sweep to the start of the next sweep's first
kernel, every host mark and every kernel (native or not) in between, in us relative to that end.

    python tools/turnaround_timeline.py MARKS.json run_kernel_trace.csv
"""
import csv
import json
import sys


def main(marks_path, trace_path):
    marks = json.load(open(marks_path))
    rows = sorted(csv.DictReader(open(trace_path)), key=lambda r: int(r["Start_Timestamp"]))
    ks = [(int(r["Start_Timestamp"]), int(r["End_Timestamp"]),
           r["Kernel_Name"].split("(")[0].replace("void ", "").replace("pfr::", "").split("<")[0][:28]) for r in rows]
    starts = [t for tag, t in marks if tag == "native_sweep_in"]
    for s0, s1 in zip(starts, starts[1:]):
        # the last kernel that ended before this step's sweep call and the first kernel after it
        ends = [e for b, e, n in ks if e < s1 and n.startswith("k_") and b > s0]
        if not ends:
            continue
        prev_end = max(ends)
        nxt = min((b, n) for b, e, n in ks if b > s1)
        ev = [(t - prev_end, tag) for tag, t in marks if prev_end - 50_000 < t <= nxt[0]]
        ev += [(b - prev_end, "kernel " + n + " (%.1f us)" % ((e - b) / 1e3)) for b, e, n in ks if prev_end <= b <= nxt[0]]
        print("step: GPU idle %.1f us" % ((nxt[0] - prev_end) / 1e3))
        for t, what in sorted(ev):
            print("   %8.1f  %s" % (t / 1e3, what))


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2])
