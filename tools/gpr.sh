#!/bin/bash
# usage: gpr.sh OUTFILE TIMEOUT CMD  -- retries only when no GPU slot/box was free (rc 3)
out=$1; shift; to=$1; shift
for i in 1 2 3 4 5 6 7 8 9 10; do
  timeout $((to + 900)) /usr/local/graft/bin/gpurun --timeout $to -- "$@" > $out 2>&1
  rc=$?
  if [ $rc -ne 3 ] && ! grep -q "status=transient" $out; then break; fi
  sleep 150
done
echo "done rc=$rc" >> $out
