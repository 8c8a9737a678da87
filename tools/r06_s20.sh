# round 6 session 20: LDS / VALU counters of the wave-uniform-key T-table microbenchmark
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/r06_v20; mkdir -p $OUT
AES_MB_TT_ONLY=1 timeout -s KILL 90 rocprofv3 --pmc SQ_INSTS_LDS SQ_INSTS_VALU SQ_LDS_IDX_ACTIVE SQ_BUSY_CYCLES SQ_WAVES SQ_LDS_BANK_CONFLICT -d $OUT/pmc -o run --output-format csv -- tools/aes_bs_mb > $OUT/mb.log 2>&1; rc=$?
python3 - $OUT <<'PY'
import csv, collections, sys, os, json
p = os.path.join(sys.argv[1], "pmc", "run_counter_collection.csv")
agg = collections.defaultdict(lambda: collections.defaultdict(float)); dur = collections.defaultdict(float); seen=set(); n=collections.Counter()
for r in csv.DictReader(open(p)):
    k = r["Kernel_Name"].split("(")[0].replace("void ", "")
    if r["Dispatch_Id"] not in seen:
        seen.add(r["Dispatch_Id"]); n[k]+=1; dur[k] += (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6
    agg[k][r["Counter_Name"]] += float(r["Counter_Value"])
out = {}
for k in agg:
    cyc = dur[k] / 1e3 * 2.4e9
    out[k] = dict(agg[k], launches=n[k], serial_ms=dur[k], lds_busy=agg[k]["SQ_LDS_IDX_ACTIVE"] / (cyc * 256) if cyc else None)
json.dump(out, open(os.path.join(sys.argv[1], "pmc_aes_ukey.json"), "w"), indent=1)
print(json.dumps(out, indent=1)[:3000])
PY
rm -rf $OUT/pmc
exit $rc
