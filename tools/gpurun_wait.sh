#!/bin/bash
# Local helper (this container): run one gpurun call; when the pool reports a transient infrastructure
# condition before the command started (no box, box lost while being prepared, back-off), wait the
# suggested time and submit the same call again (up to 8 times).  A call whose command ran is never
# resubmitted.  usage: gpurun_wait.sh LOGFILE TIMEOUT 'command'
LOG=$1; TO=$2; shift 2
for i in 1 2 3 4 5 6 7 8; do
  /usr/local/graft/bin/gpurun --timeout $TO -- "$@" > $LOG 2>&1
  rc=$?
  if grep -q "status=transient" $LOG && grep -Eq "run 0.0s|run Nones" $LOG; then
    w=$(grep -oE "retry in [0-9]+s" $LOG | grep -oE "[0-9]+" | head -1)
    w=${w:-120}
    echo "[wait] transient (attempt $i), sleeping $((w + 10)) s" >> $LOG.attempts
    sleep $((w + 10))
    continue
  fi
  exit $rc
done
exit 3
