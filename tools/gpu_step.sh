#!/bin/bash
# Run one GPU step with a time limit; return 0 if it passed or merely had failing tests (rc 1),
# stop the whole script on a crash / timeout (124, 134, 137, 139, …).
#   source tools/gpu_step.sh; step NAME SECONDS cmd...
step() {
  local name=$1 secs=$2; shift 2
  echo "[step] $name" >&2
  set +e
  timeout -k 10 "$secs" "$@"
  local rc=$?
  set -e
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "[step] $name: rc $rc — stopping"; exit $rc; fi
  echo "[step] $name: rc $rc" >&2
}
