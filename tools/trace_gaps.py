"""Where a sweep's GPU time goes outside its level kernels, from a rocprofv3
--kernel-trace CSV (run_kernel_trace.csv).

    python tools/trace_gaps.py <run_kernel_trace.csv> [--split-gap-ms G | --split-after K] [--from-ms A]
                               [--to-ms B] [--last N]

The trace is cut into segments at host gaps longer than G ms, or after every
launch of kernel K (e.g. k_decide: one segment per sweep level, both
aggregators' prep_init and decide).  Per segment: its wall time, the union of the level-kernel launches
(k_eval_aes*, k_node_proof), and the rest of the wall split into time when
some other kernel runs (attributed to the kernels running then, each share
being the time that kernel alone covers, overlaps split evenly) and idle
time.  --last N keeps the last N segments (the timed sweep).  Not part of the
product."""
import argparse
import collections

from trace_summary import load, short

LEVEL = ("k_eval_aes", "k_node_proof")


def union(iv):
    out = []
    for (s, e) in sorted(iv):
        if out and s <= out[-1][1]:
            out[-1][1] = max(out[-1][1], e)
        else:
            out.append([s, e])
    return out


def minus(a, b):
    """a - b for sorted disjoint interval lists."""
    out, j = [], 0
    for (s, e) in a:
        cur = s
        while j < len(b) and b[j][1] <= cur:
            j += 1
        k = j
        while k < len(b) and b[k][0] < e:
            if b[k][0] > cur:
                out.append([cur, b[k][0]])
            cur = max(cur, b[k][1])
            k += 1
        if cur < e:
            out.append([cur, e])
    return out


def length(iv):
    return sum(e - s for (s, e) in iv)


def segment(rows):
    lo, hi = rows[0][0], max(r[1] for r in rows)
    lvl = union([(s, e) for (s, e, n) in rows if short(n).startswith(LEVEL)])
    rest = minus([[lo, hi]], lvl)
    # sweep over event boundaries inside `rest`, splitting each slice among the
    # kernels running in it
    ev = []
    for (s, e, n) in rows:
        k = short(n)
        if k.startswith(LEVEL):
            continue
        ev.append((s, 1, k))
        ev.append((e, -1, k))
    ev.sort(key=lambda x: (x[0], x[1]))
    per = collections.defaultdict(float)
    running = collections.Counter()
    t_prev = None
    idle = 0.0
    for (t, d, k) in ev + [(hi, 0, None)]:
        if t_prev is not None and t > t_prev:
            sl = length(minus([[t_prev, t]], lvl))
            act = [x for (x, c) in running.items() if c > 0]
            if act:
                for x in act:
                    per[x] += sl / len(act)
            else:
                idle += sl
        if k is not None:
            running[k] += d
        t_prev = t if t_prev is None else max(t_prev, t)
    # time before the first non-level event and outside level kernels
    covered = sum(per.values()) + idle
    idle += max(0.0, length(rest) - covered)
    return hi - lo, length(lvl), per, idle


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--split-gap-ms", type=float, default=2.0)
    ap.add_argument("--split-after", default="")
    ap.add_argument("--from-ms", type=float, default=0.0)
    ap.add_argument("--to-ms", type=float, default=1e18)
    ap.add_argument("--last", type=int, default=0)
    a = ap.parse_args()
    rows = [r for r in load(a.trace) if r[0] >= a.from_ms and r[1] <= a.to_ms]
    segs, seg, last_end = [], [], None
    for r in rows:
        if not a.split_after and last_end is not None and r[0] - last_end > a.split_gap_ms:
            segs.append(seg)
            seg = []
        seg.append(r)
        last_end = max(last_end or 0.0, r[1])
        if a.split_after and short(r[2]).startswith(a.split_after):
            segs.append(seg)
            seg = []
    if seg:
        segs.append(seg)
    if a.last:
        segs = segs[-a.last:]
    tot = collections.defaultdict(float)
    (tw, tl, ti) = (0.0, 0.0, 0.0)
    for (i, sg) in enumerate(segs):
        (wall, lvl, per, idle) = segment(sg)
        tw += wall
        tl += lvl
        ti += idle
        for (k, v) in per.items():
            tot[k] += v
        top = sorted(per.items(), key=lambda kv: -kv[1])[:3]
        print("seg %3d wall %8.2f level %8.2f other %7.2f idle %6.2f  %s" % (
            i, wall, lvl, sum(per.values()), idle, "  ".join("%s %.2f" % kv for kv in top)))
    print("total: wall %.2f ms, level kernels %.2f ms, outside them %.2f ms (kernels %.2f, idle %.2f)" % (
        tw, tl, tw - tl, sum(tot.values()), ti))
    for (k, v) in sorted(tot.items(), key=lambda kv: -kv[1]):
        print("  %-36s %9.2f ms" % (k, v))


if __name__ == "__main__":
    main()
