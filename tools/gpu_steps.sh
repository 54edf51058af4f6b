#!/bin/bash
# Runs GPU steps in order, each under its own time limit, logging to
# gpurun_out/<name>.log.  A step that fails normally (exit 1: test failures)
# does not stop the sequence; a crash, abort, timeout or signal (exit >= 2)
# stops it: nothing else touches the GPU after that.
#   tools/gpu_steps.sh NAME SECONDS 'COMMAND' [NAME SECONDS 'COMMAND' ...]
set -u
mkdir -p gpurun_out
while [ $# -ge 3 ]; do
  name=$1; secs=$2; cmd=$3; shift 3
  mkdir -p "gpurun_out/$(dirname "$name")"
  echo "== $name (limit ${secs}s): $cmd"
  timeout -k 10 "$secs" bash -c "$cmd" > "gpurun_out/$name.log" 2>&1
  rc=$?
  echo "== $name rc=$rc"; tail -n 5 "gpurun_out/$name.log"
  if [ $rc -ge 2 ]; then echo "== stopping after $name (rc=$rc)"; exit $rc; fi
done
