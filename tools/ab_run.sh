#!/bin/bash
# A/B timing on one GPU box (run through gpurun from the repo root):
#   tools/ab_run.sh <tag> <reps> <variant> [<variant> ...]
# variant = name|ENV=V,ENV=V|config|extra+bench+args   (fields may be empty;
# LIB=build/lib....so selects another build of the library: bench.py --lib).
# Variants run interleaved <reps> times (A B A B ...) so box drift hits all
# alike; each run under its own time limit; a failure ends the script.
# Output: gpurun_out/<tag>/<name>_<rep>.json (+ .log), summary.txt
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
TAG=$1; REPS=$2; shift 2
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
for rep in $(seq 1 "$REPS"); do
    for v in "$@"; do
        IFS='|' read -r name envs cfg args <<< "$v"
        cfg=${cfg:-c2}
        args=${args//+/ }
        envarr=()
        lib=()
        if [ -n "$envs" ]; then IFS=',' read -r -a ev <<< "$envs"; fi
        for e in "${ev[@]}"; do
            case $e in LIB=*) lib=(--lib "$PWD/${e#LIB=}") ;; *) envarr+=("$e") ;; esac
        done
        unset ev
        echo "[$(date +%T)] $name rep $rep: ${envarr[*]} bench --config $cfg $args ${lib[*]}" >> "$OUT/steps.txt"
        env "${envarr[@]}" timeout -k 10 300 python3 -u bench.py --config "$cfg" --cpu-baseline 0 --full-job 0 $args "${lib[@]}" \
            > "$OUT/${name}_$rep.log" 2>&1
        rc=$?
        if [ $rc -ne 0 ]; then echo "$name rc=$rc" >> "$OUT/steps.txt"; tail -20 "$OUT/${name}_$rep.log"; exit $rc; fi
        tail -1 "$OUT/${name}_$rep.log" > "$OUT/${name}_$rep.json"
        python3 - "$OUT/${name}_$rep.json" "$name" >> "$OUT/summary.txt" <<'EOF'
import json, sys
d = json.load(open(sys.argv[1]))
b = d.get("breakdown_ms_per_step", {})
print("%-16s %9.4g %s  frac %.3f  eval %7.1f  absorb %7.1f  step %7.1f" % (
    sys.argv[2], d["value"], d["unit"], d.get("roofline", {}).get("frac", 0),
    b.get("eval_aes", b.get("eval_aes_plus_proofs", 0)), b.get("absorb", 0), d["ms_per_step"]))
EOF
    done
done
cat "$OUT/summary.txt"
echo done >> "$OUT/steps.txt"
