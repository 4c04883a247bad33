#!/bin/bash
# GPU-box driver: runs named steps, each under its own time limit, logs under
# gpurun_out/$TAG/.  A step that fails with an ordinary error (rc 1) does not
# stop the next ones; a fault, abort, segfault or time limit ends the call.
# usage: TAG=r03a bash tools/gpu_run.sh "name|limit_s|command" ...
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-run}
mkdir -p "$OUT"
for spec in "$@"; do
    name=${spec%%|*}; rest=${spec#*|}; lim=${rest%%|*}; cmd=${rest#*|}
    t0=$(date +%s)
    timeout -k 10 "$lim" bash -c "$cmd" > "$OUT/$name.log" 2>&1
    rc=$?
    echo "$name rc=$rc $(( $(date +%s) - t0 ))s"
    tail -3 "$OUT/$name.log"
    if [ $rc -ne 0 ] && { [ $rc -ne 1 ] || [ "${STRICT:-0}" = 1 ]; }; then echo "stopping after $name (rc $rc)"; exit $rc; fi
done
