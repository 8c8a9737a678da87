"""Add or replace one (config, prefixes, reports) entry of profiles/eval_traffic.json (the HBM bytes bench.py reports as
roofline.traffic) with the FETCH_SIZE / WRITE_SIZE passes of a tools/gpu_session.sh pmc:<cfg> run.

    python tools/update_eval_traffic.py <pmc_summary.json> <cfg> <reports> <prefixes> <kernel> <tag>

<pmc_summary.json> is tools/pmc_summary.py's output for that run (one timed step)."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def main(summary, cfg, reports, prefixes, kernel, tag):
    s = json.load(open(summary))[kernel]
    path = os.path.join(ROOT, "profiles", "eval_traffic.json")
    d = json.load(open(path))
    rd, wr, n = s["hbm_read_bytes"], s["hbm_write_bytes"], s["launches"]
    entry = {
        "config": cfg, "kernel": kernel, "reports": int(reports), "prefixes": int(prefixes),
        "launches_per_step": n, "hbm_read_bytes_per_step": rd, "hbm_write_bytes_per_step": wr,
        "hbm_bytes_per_launch": (rd + wr) / n, "serial_ms_per_step": s["serial_ms"],
        "hbm_gbs_serialized": (rd + wr) / (s["serial_ms"] / 1e3) / 1e9,
        "measured": "%s (%s)" % (tag, os.path.relpath(summary, ROOT)),
    }
    # one entry per (config, prefixes, reports): measurements at other batch sizes stay
    d["entries"] = [e for e in d["entries"]
                    if (e["config"], e["prefixes"], e["reports"]) != (cfg, int(prefixes), int(reports))] + [entry]
    json.dump(d, open(path, "w"), indent=1)
    print(json.dumps(entry, indent=1))


if __name__ == "__main__":
    main(*sys.argv[1:7])
