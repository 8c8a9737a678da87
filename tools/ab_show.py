import glob, json, os
for f in sorted(glob.glob(os.path.join(os.path.dirname(__file__), "..", "gpurun_out", "ab_*.json"))):
    try:
        d = json.load(open(f))
    except Exception as e:
        print(os.path.basename(f), "unreadable", e)
        continue
    b = d["breakdown_ms_per_step"]
    print("%-28s %6.1f M/s  eval %5.0f  np %5.0f  abs %5.0f  tot %5.0f" % (
        os.path.basename(f), d["value"] / 1e6, b["eval_aes"], b.get("node_proof", b.get("node_proof_last_level", 0)), b["absorb"], b["prep_init_total"]))
