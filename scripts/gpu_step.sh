#!/bin/bash
# Shared helper for GPU command scripts: step <name> <seconds> <cmd...> runs one GPU step under its own time limit,
# logs to gpurun_out/<name>.log, prints rc + tail, and stops the script at the first failure.
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out
step() {
  local name=$1 secs=$2; shift 2
  timeout -k 10 "$secs" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "$name rc=$rc"; tail -${TAILN:-4} "gpurun_out/$name.log"
  [ $rc -eq 0 ] || exit $rc
}
