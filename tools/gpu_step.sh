#!/bin/bash
# Runs one GPU step under its own time limit; stops the whole script on a fault/abort/timeout.
# usage: gpu_step.sh SECONDS LOGFILE cmd...
secs=$1; log=$2; shift 2
timeout -k 10 "$secs" "$@" > "$log" 2>&1
rc=$?
echo "[gpu_step] rc=$rc : $*" >> "$log"
case $rc in
  0) exit 0 ;;
  1|2|3|4|5) exit 1 ;;            # ordinary failure (python exception / test failure)
  *) echo "FATAL rc=$rc ($*) -- stopping" >&2; exit 99 ;;
esac
