#!/bin/bash
# usage: gpurun_retry.sh <logfile> <timeout> <command...>; retries only when the box never ran the command
# Retries only "transient" outcomes (the box never ran the command; nothing charged).
LOG=$1; shift; TO=$1; shift
for i in 1 2 3 4 5 6 7 8 9 10; do
  /usr/local/graft/bin/gpurun --timeout $TO -- "$@" > $LOG 2>&1
  rc=$?
  if grep -q "status=transient\|no box or slot" $LOG && ! grep -q "run [1-9]" $LOG; then
    echo "[retry $i: transient]" >> $LOG.retries; sleep 120; continue
  fi
  exit $rc
done
