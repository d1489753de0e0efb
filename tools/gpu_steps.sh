#!/usr/bin/env bash
# Run GPU steps in order, each under its own time limit; logs go to gpurun_out/<name>.log.
# A step that fails normally (exit 1, e.g. a failing test) does not stop the chain; a fault,
# abort, segfault, kill or timeout (any other non-zero code) ends the script immediately
# (no further GPU work after a fault).
#   usage: tools/gpu_steps.sh "name|seconds|command" ...
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
worst=0
for spec in "$@"; do
  name="${spec%%|*}"; rest="${spec#*|}"; secs="${rest%%|*}"; cmd="${rest#*|}"
  echo "=== [$name] ($secs s): $cmd"
  start=$(date +%s)
  timeout -k 10 "$secs" bash -c "$cmd" > "gpurun_out/$name.log" 2>&1
  rc=$?
  echo "=== [$name] rc=$rc in $(( $(date +%s) - start )) s"
  tail -n 15 "gpurun_out/$name.log"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "=== stopping after [$name] (rc=$rc)"; exit $rc; fi
  [ $rc -gt $worst ] && worst=$rc
done
exit $worst
