# round 6 session 5: same-box A/B of the small-level split cost model (choose_split with the proof
# waves' head start) on the north_star sweep, then the binder sponges standalone (knob build,
# MASTIC_SERIAL_SPONGES=1) for C2, C5 and the north_star sweep, then a PMC pass of the sponge kernels
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/r06_v5; mkdir -p $OUT
run() { local name=$1 t=$2; shift 2; echo "[$(date +%T)] $name" >> $OUT/steps.txt
        timeout -k 10 $t "$@" > $OUT/$name.log 2>&1; local rc=$?; echo "[$(date +%T)] $name rc=$rc" >> $OUT/steps.txt
        tail -1 $OUT/$name.log | cut -c1-300; [ $rc -ne 0 ] && exit $rc; return 0; }
SW="--config c2sweep --steps 1 --warmup 1 --cpu-baseline 0"
run ab_new1 300 python3 -u bench.py $SW
run ab_old1 300 python3 -u bench.py $SW --lib build/libmastic_r05final.so
run ab_new2 300 python3 -u bench.py $SW
run ab_old2 300 python3 -u bench.py $SW --lib build/libmastic_r05final.so
export MASTIC_SERIAL_SPONGES=1
run serial_c2 300 python3 -u bench.py --config c2 --steps 2 --north-star 0 --full-job 0 --cpu-baseline 0 --lib build/libmastic_knobs.so
run serial_c5 300 python3 -u bench.py --config c5 --steps 2 --full-job 0 --cpu-baseline 0 --lib build/libmastic_knobs.so
run serial_c2sweep 400 python3 -u bench.py $SW --lib build/libmastic_knobs.so
unset MASTIC_SERIAL_SPONGES
run pmc_c2 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_BUSY_CYCLES -d $OUT/pmc_c2 -o run --output-format csv -- python3 bench.py --config c2 --steps 1 --warmup 0 --north-star 0 --full-job 0 --cpu-baseline 0
run pmc_c2sweep 400 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_BUSY_CYCLES -d $OUT/pmc_c2sweep -o run --output-format csv -- python3 bench.py --config c2sweep --reports 131072 --steps 1 --warmup 0 --cpu-baseline 0
python3 - $OUT <<'PY'
import csv, collections, json, sys, os
out = {}
for tag in ("c2", "c2sweep"):
    p = os.path.join(sys.argv[1], "pmc_%s" % tag, "run_counter_collection.csv")
    if not os.path.exists(p):
        continue
    agg = collections.defaultdict(lambda: collections.defaultdict(float)); n = collections.Counter(); dur = collections.defaultdict(float); seen = set()
    for r in csv.DictReader(open(p)):
        k = r["Kernel_Name"].split("(")[0].replace("void ", "").split("<")[0]
        if r["Dispatch_Id"] not in seen:
            seen.add(r["Dispatch_Id"]); n[k] += 1
            dur[k] += (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6
        agg[k][r["Counter_Name"]] += float(r["Counter_Value"])
    out[tag] = {k: dict(agg[k], launches=n[k], serial_ms=dur[k]) for k in agg if k.startswith("k_absorb") or k.startswith("k_eval") or k == "k_node_proof"}
json.dump(out, open(os.path.join(sys.argv[1], "pmc_sponges.json"), "w"), indent=1)
PY
rm -rf $OUT/pmc_c2 $OUT/pmc_c2sweep
echo done >> $OUT/steps.txt
