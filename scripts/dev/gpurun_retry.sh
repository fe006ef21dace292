#!/bin/bash
# gpurun_retry.sh OUT TIMEOUT 'COMMAND' -- submit one gpurun call, and while
# the pool has no box for it (gpurun exit 3 / "backing off": nothing ran,
# nothing charged) wait and submit it again, at most 30 times.  A call that
# RAN is never repeated, whatever its result.
out=$1; to=$2; cmd=$3
for i in $(seq 1 30); do
  /usr/local/graft/bin/gpurun --timeout "$to" -- "$cmd" > "$out" 2>&1
  rc=$?
  if [ $rc -ne 3 ] && ! grep -q "backing off\|no free box" "$out"; then
    echo "gpurun rc=$rc after $i submission(s)" >> "$out"
    exit $rc
  fi
  sleep 150
done
echo "gave up: no box after 30 submissions" >> "$out"
exit 3
