#!/bin/bash
# gpurun with retries on "no box / slot free" and harness transients only (never on a command failure)
# usage: gpr.sh <logfile> <timeout> <command>
LOG=$1; TO=$2; shift 2
for i in $(seq 1 12); do
  timeout $((TO + 1500)) /usr/local/graft/bin/gpurun --timeout $TO -- "$@" > $LOG 2>&1
  rc=$?
  if grep -q "status=transient\|no free box\|slot(s) on this pod are busy" $LOG && ! grep -q "status=ok" $LOG; then
    echo "[gpr] attempt $i: transient/no slot, retrying in 150 s" >> $LOG.retries
    sleep 150
    continue
  fi
  break
done
echo "done rc=$rc" >> $LOG
