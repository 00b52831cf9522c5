"""Reconcile a rocprofv3 kernel trace with bench.py's ms_per_step.

    python scripts/reconcile_trace.py <run_kernel_trace.csv> <marker regex> [bench json]

Splits the trace into step windows at each launch of the marker kernel (the step's first
kernel), keeps the windows whose launch sequence is the modal one (the graph replays of
the timed leg), and prints per window: wall (marker to next marker), busy (sum of kernel
durations), the sum of the gaps between consecutive kernels, and the kernel count.  With
the bench JSON of an untraced run, also the tracer's cost: traced wall - untraced
ms_per_step, split into gaps (dispatch / completion-signal overhead between kernels) and
duration inflation (busy - the untraced step)."""
import csv
import json
import re
import statistics
import sys


def windows(path, marker):
    rows = []
    with open(path) as f:
        for r in csv.DictReader(f):
            rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]))
    rows.sort()
    pat = re.compile(marker)
    idx = [i for i, r in enumerate(rows) if pat.search(r[2])]
    out = []
    for a, b in zip(idx, idx[1:]):
        w = rows[a:b]
        names = tuple(re.sub(r"\(.*", "", n)[:60] for _, _, n in w)
        busy = sum(e - s for s, e, _ in w)
        # idle time between consecutive kernels, the last one to the next step's marker
        # included (overlapping launches count 0)
        ends = [e for _, e, _ in w] + [None]
        starts = [s for s, _, _ in w[1:]] + [rows[b][0]]
        gaps = sum(max(0, st - en) for st, en in zip(starts, ends))
        out.append(dict(wall=rows[b][0] - w[0][0], busy=busy, gaps=gaps, n=len(w), seq=names))
    return out


def main():
    path, marker = sys.argv[1], sys.argv[2]
    ws = windows(path, marker)
    if not ws:
        sys.exit("no marker launches in the trace")
    modal = statistics.mode(w["seq"] for w in ws)
    sel = [w for w in ws if w["seq"] == modal]
    med = {k: statistics.median(w[k] for w in sel) / 1e3 for k in ("wall", "busy", "gaps")}
    res = {"windows": len(sel), "kernels_per_step": len(modal),
           "traced_wall_us": round(med["wall"], 1), "busy_us": round(med["busy"], 1),
           "gaps_us": round(med["gaps"], 1),
           "gap_per_kernel_us": round(med["gaps"] / len(modal), 2)}
    if len(sys.argv) > 3:
        for line in open(sys.argv[3]):
            if line.startswith("{"):
                untraced = json.loads(line)["ms_per_step"] * 1e3
                res["untraced_ms_per_step_us"] = round(untraced, 1)
                res["tracer_cost_us"] = round(med["wall"] - untraced, 1)
                res["busy_minus_untraced_us"] = round(med["busy"] - untraced, 1)
                break
    print(json.dumps(res))


if __name__ == "__main__":
    main()
