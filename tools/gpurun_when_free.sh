#!/bin/bash
# Run one gpurun command, waiting for a free box: retries ONLY when gpurun
# reports that nothing ran (status "transient": no box / slot free, or the box
# failed while being prepared; nothing charged).  A command that ran, whatever
# its outcome, is never retried.
#   tools/gpurun_when_free.sh <timeout_s> '<command>'
t="$1"; shift
for i in $(seq 1 20); do
    /usr/local/graft/bin/gpurun --timeout "$t" -- "$@"
    rc=$?
    st=$(python3 -c "import json;d=json.load(open('/root/repo/gpurun_out/.last_call.json'));print(d.get('status'), d.get('run_s'))" 2>/dev/null)
    case "$st" in
        "transient 0.0"|"transient 0") echo "[when_free] nothing ran ($st), waiting"; sleep 150 ;;
        *) exit $rc ;;
    esac
done
exit $rc
