#!/bin/bash
# Run GPU steps in order, each under its own time limit, logging to gpurun_out/<name>.log.
# usage: scripts/gpu_steps.sh name1 secs1 'cmd1' [name2 secs2 'cmd2' ...]
# A step that faults, aborts, segfaults or times out (exit >= 124) ends the chain: nothing else
# touches the GPU in this call. An ordinary failure (e.g. pytest exit 1) is logged and the
# chain continues.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
mkdir -p gpurun_out
export TMPDIR=/tmp
rc_all=0
while [ $# -ge 3 ]; do
  name=$1; secs=$2; cmd=$3; shift 3
  echo "=== $name (limit ${secs}s): $cmd" | tee -a gpurun_out/steps.log
  start=$(date +%s)
  timeout -k 10 "$secs" bash -c "$cmd" > "gpurun_out/$name.log" 2>&1
  rc=$?
  echo "=== $name rc=$rc in $(( $(date +%s) - start ))s" | tee -a gpurun_out/steps.log
  tail -n 5 "gpurun_out/$name.log"
  if [ $rc -ge 124 ] || [ $rc -eq 134 ] || [ $rc -eq 139 ]; then
    echo "=== fatal exit $rc: stopping the chain" | tee -a gpurun_out/steps.log
    exit $rc
  fi
  [ $rc -ne 0 ] && rc_all=$rc
done
exit $rc_all
