"""Summarise a rocprofv3 --kernel-trace CSV (run_kernel_trace.csv) over a time
window: per kernel the launches and summed duration, the union of busy time
(all queues) against the window's wall time, and the idle gaps.

    python tools/trace_summary.py <run_kernel_trace.csv> [--from-ms A] [--to-ms B] [--split-gap-ms G]

Times are relative to the first dispatch.  --split-gap-ms G prints, instead of
one window, one line per segment separated by host gaps longer than G ms (the
sweep's levels are separated by the host's pruning round trip).  Not part of
the product."""
import argparse
import collections
import csv


def load(path):
    rows = []
    with open(path) as f:
        for r in csv.DictReader(f):
            rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]))
    rows.sort()
    t0 = rows[0][0]
    return [((s - t0) / 1e6, (e - t0) / 1e6, n) for (s, e, n) in rows]


def short(name):
    return name.split("(")[0].replace("void ", "")


def summarise(rows, lo, hi):
    sel = [r for r in rows if r[0] >= lo and r[1] <= hi]
    if not sel:
        return None
    per = collections.defaultdict(lambda: [0, 0.0])
    for (s, e, n) in sel:
        per[short(n)][0] += 1
        per[short(n)][1] += e - s
    busy, cur_s, cur_e = 0.0, None, None
    for (s, e, _n) in sel:
        if cur_e is None or s > cur_e:
            if cur_e is not None:
                busy += cur_e - cur_s
            cur_s, cur_e = s, e
        else:
            cur_e = max(cur_e, e)
    busy += cur_e - cur_s
    wall = sel[-1][1] - sel[0][0]
    return per, busy, wall, sel[0][0], sel[-1][1]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--from-ms", type=float, default=0.0)
    ap.add_argument("--to-ms", type=float, default=1e18)
    ap.add_argument("--split-gap-ms", type=float, default=0.0)
    a = ap.parse_args()
    rows = load(a.trace)
    if a.split_gap_ms > 0:
        seg, segs = [], []
        last_end = None
        for r in rows:
            if r[0] < a.from_ms or r[1] > a.to_ms:
                continue
            if last_end is not None and r[0] - last_end > a.split_gap_ms:
                segs.append(seg)
                seg = []
            seg.append(r)
            last_end = max(last_end or 0.0, r[1])
        if seg:
            segs.append(seg)
        for (i, sg) in enumerate(segs):
            per, busy, wall, s, e = summarise(sg, -1, 1e18)
            top = sorted(per.items(), key=lambda kv: -kv[1][1])[:4]
            print("seg %3d  %9.2f-%9.2f ms  wall %8.2f  busy %8.2f  %s" % (
                i, s, e, wall, busy, "  ".join("%s %d/%.2f" % (k, v[0], v[1]) for (k, v) in top)))
        return
    res = summarise(rows, a.from_ms, a.to_ms)
    per, busy, wall, s, e = res
    print("window %.2f-%.2f ms: wall %.2f ms, GPU busy %.2f ms (%.1f %%), idle %.2f ms" % (
        s, e, wall, busy, 100 * busy / wall, wall - busy))
    for (k, v) in sorted(per.items(), key=lambda kv: -kv[1][1]):
        print("  %-40s %7d launches %11.2f ms  (%5.1f %% of busy)" % (k, v[0], v[1], 100 * v[1] / busy))


if __name__ == "__main__":
    main()
