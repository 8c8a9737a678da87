"""Summarise a tools/profile_r01.sh output directory: per-kernel serialized
duration (PMC passes), VALU / LDS utilisation, wave-state split, HBM bytes."""
import collections
import csv
import json
import os
import sys

CLK = 2.4e9
CUS = 256


def load(path):
    rows = list(csv.DictReader(open(path)))
    dur = collections.defaultdict(float)
    n = collections.Counter()
    seen = set()
    vals = collections.defaultdict(lambda: collections.defaultdict(float))
    for r in rows:
        k = r["Kernel_Name"].split("(")[0].replace("void ", "")
        fc = ",FC" if "true, true" in k else ""  # the frontier-cache instantiation (hits, a cache-on last level)
        k = k.split("<")[0] + ("<F128%s>" % fc if "F128" in k else "<F64%s>" % fc if "F64" in k else "")
        if r["Dispatch_Id"] not in seen:
            seen.add(r["Dispatch_Id"])
            dur[k] += (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6
            n[k] += 1
        vals[k][r["Counter_Name"]] += float(r["Counter_Value"])
    return dur, n, vals


def main(d, suffix="", kernels=("k_eval_aes<F64>", "k_eval_aes<F128>", "k_eval_aes<F64,FC>", "k_eval_aes<F128,FC>",
                                 "k_node_proof", "k_absorb_pair", "k_absorb", "k_fold<F64>", "k_fold<F128>")):
    """d: the output directory; suffix: "_<cfg>" for tools/gpu_session.sh pmc:<cfg> passes."""
    out = {}
    dur, n, sq1 = load(os.path.join(d, "sq1%s/run_counter_collection.csv" % suffix))
    _, _, sq2 = load(os.path.join(d, "sq2%s/run_counter_collection.csv" % suffix))
    _, _, fe = load(os.path.join(d, "fetch%s/run_counter_collection.csv" % suffix))
    _, _, wr = load(os.path.join(d, "write%s/run_counter_collection.csv" % suffix))
    for k in kernels:
        if k not in dur:
            continue
        ms = dur[k]
        cyc = ms / 1e3 * CLK
        v1, v2 = sq1[k], sq2[k]
        act = v2["SQ_ACTIVE_INST_ANY"] or 1.0
        out[k] = {
            "launches": n[k],
            "serial_ms": ms,
            # wave64 VALU issue: 2 cycles per instruction on a SIMD for full-rate ops
            # (v_xor/v_bitop3/v_add), 4 for half-rate ones (v_perm/v_alignbit/v_bfe/...):
            # profiles/r01_v9_valu_peak.json (tools/valu_peak.hip).  The two bounds:
            "valu_busy_if_all_full_rate": v1["SQ_INSTS_VALU"] * 2 / (cyc * CUS * 4),
            "valu_busy_if_all_half_rate": v1["SQ_INSTS_VALU"] * 4 / (cyc * CUS * 4),
            "lds_busy": v2["SQ_LDS_IDX_ACTIVE"] / (cyc * CUS),
            "wait_any_over_active": v2["SQ_WAIT_ANY"] / act,
            "wait_inst_any_over_active": v2["SQ_WAIT_INST_ANY"] / act,
            "wait_inst_lds_over_active": v2["SQ_WAIT_INST_LDS"] / act,
            "valu_wave_instr": v1["SQ_INSTS_VALU"],
            "lds_wave_instr": v1["SQ_INSTS_LDS"],
            "hbm_read_bytes": 2 * fe[k]["FETCH_SIZE"] * 1024,  # KB units; gfx950 counts half (MI355X_MICROARCH.md)
            "hbm_write_bytes": wr[k]["WRITE_SIZE"] * 1024,
        }
    return out


if __name__ == "__main__":
    print(json.dumps(main(sys.argv[1], sys.argv[2] if len(sys.argv) > 2 else ""), indent=1))
