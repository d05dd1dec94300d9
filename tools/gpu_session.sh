#!/bin/bash
# Runs a sequence of GPU steps on the gpurun box, each under its own time limit.
# A test FAILURE (exit 1) lets later steps run; a crash, abort, fault or time-out
# (124, 134, 137, 139, >128) ends the session immediately.
# usage: tools/gpu_session.sh "<seconds> <command...>" ...
mkdir -p gpurun_out
export TMPDIR=/tmp
for spec in "$@"; do
  secs=${spec%% *}
  cmd=${spec#* }
  echo "=== [$(date +%T)] ($secs s) $cmd" | tee -a gpurun_out/session.log
  timeout -k 10 "$secs" bash -c "$cmd" >> gpurun_out/session.log 2>&1
  rc=$?
  echo "=== rc=$rc" | tee -a gpurun_out/session.log
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then
    echo "stopping session after rc=$rc" | tee -a gpurun_out/session.log
    exit $rc
  fi
done
exit 0
