#!/bin/bash
# gpurun with retries ONLY when no box was obtained (status=transient / exit 3:
# nothing ran).  Usage: tools/gr.sh <timeout> '<command>'   (log: gpurun_out/gr.txt)
T=$1; shift
for i in 1 2 3 4 5 6; do
  /usr/local/graft/bin/gpurun --timeout "$T" -- "$@" > gpurun_out/gr.txt 2>&1
  rc=$?
  if grep -q "status=transient" gpurun_out/gr.txt || [ $rc -eq 3 ]; then
    echo "transient (try $i), waiting" >&2; sleep 45; continue
  fi
  break
done
grep -E "status=|GPU-minutes" gpurun_out/gr.txt
exit $rc
