#!/bin/bash
# Run GPU steps in sequence; stop at the first step that faults / aborts / times out.
# usage: tools/gpu_run.sh "<name>:<timeout_s>:<command>" ...
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for spec in "$@"; do
  name="${spec%%:*}"; rest="${spec#*:}"; tmo="${rest%%:*}"; cmd="${rest#*:}"
  echo "=== $name (timeout ${tmo}s): $cmd" | tee -a gpurun_out/steps.log
  timeout -k 10 "$tmo" bash -c "$cmd" > "gpurun_out/$name.log" 2>&1
  rc=$?
  echo "=== $name rc=$rc" | tee -a gpurun_out/steps.log
  tail -5 "gpurun_out/$name.log"
  case $rc in
    0|1|2|5) ;;                       # success / test failures / usage: keep going
    *) echo "stopping after $name (rc=$rc)"; exit $rc ;;
  esac
done
