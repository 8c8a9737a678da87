"""Summarise rocprofv3 kernel traces of the level kernel (k_eval_aes):
  python3 tools/level_trace_summary.py sweep <run_kernel_trace.csv>
      launches by duration class (the tiny top tree levels vs the rest)
  python3 tools/level_trace_summary.py probe <dir with variant subdirs> <levels>
      tools/tiny_level_probe.py runs: the last rep's per-level launch
      durations for each knob variant (base, noaes, noproof, nosplit, nosponge)
"""
import collections
import csv
import os
import sys


def load(path):
    out = []
    for r in csv.DictReader(open(path)):
        if "k_eval_aes" not in r["Kernel_Name"]:
            continue
        name = r["Kernel_Name"].split("(")[0].replace("void ", "")
        out.append((name, (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3, int(r["Grid_Size_X"])))
    return out


def sweep(path):
    ev = load(path)
    total = sum(d for (_, d, _) in ev)
    print("%d k_eval_aes launches, %.1f ms" % (len(ev), total / 1e3))
    for (lo, hi) in ((0, 1000), (1000, 5000), (5000, 20000), (20000, 1e12)):
        sel = [d for (_, d, _) in ev if lo <= d < hi]
        print("  launches of %6.0f-%-8s us: %5d, %9.1f ms (%.1f %% of the level-kernel time)" %
              (lo, "inf" if hi == 1e12 else "%.0f" % hi, len(sel), sum(sel) / 1e3, 100 * sum(sel) / total))
    by = collections.defaultdict(lambda: [0, 0.0])
    for (n, d, _) in ev:
        by[n][0] += 1
        by[n][1] += d
    for (n, (c, d)) in sorted(by.items(), key=lambda kv: -kv[1][1]):
        print("  %-45s %5d launches %9.1f ms" % (n, c, d / 1e3))


def probe(root, levels):
    print("last rep, per-level k_eval_aes launch durations (us), levels 0..%d" % (levels - 1))
    for v in sorted(os.listdir(root)):
        p = os.path.join(root, v, "run_kernel_trace.csv")
        if not os.path.exists(p):
            continue
        ev = load(p)[-levels:]
        print("  %-9s %s  sum %.0f" % (v, " ".join("%6.0f" % d for (_, d, _) in ev), sum(d for (_, d, _) in ev)))


if __name__ == "__main__":
    if sys.argv[1] == "sweep":
        sweep(sys.argv[2])
    else:
        probe(sys.argv[2], int(sys.argv[3]))
