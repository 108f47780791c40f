#!/bin/bash
# Runs GPU steps in order, each under its own time limit; stops at the first
# step that timed out, aborted or crashed (exit status 124, 134, 137, 139 or
# > 128), continues past ordinary failures (pytest's 1).
#   tools/gpu_steps.sh "SECONDS LOG -- CMD..." ...
# Every step's status goes to gpurun_out/steps.txt.
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
: > gpurun_out/steps.txt
worst=0
for step in "$@"; do
  secs=${step%% *}; rest=${step#* }
  log=${rest%% -- *}; cmd=${rest#* -- }
  start=$(date +%s)
  timeout -k 10 "$secs" bash -c "$cmd" > "gpurun_out/$log" 2>&1
  rc=$?
  echo "rc=$rc ${secs}s-limit $(( $(date +%s) - start ))s $log: $cmd" >> gpurun_out/steps.txt
  tail -2 "gpurun_out/$log" | sed 's/^/    /' >> gpurun_out/steps.txt
  [ $rc -ne 0 ] && worst=$rc
  if [ $rc -eq 124 ] || [ $rc -gt 128 ]; then echo "stopping after $log (rc=$rc)" >> gpurun_out/steps.txt; exit $rc; fi
done
exit $worst
