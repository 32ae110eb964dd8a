#!/bin/bash
# Submit one gpurun call, waiting while no GPU slot is free (gpurun exit 3: nothing ran, nothing
# charged) or the box could not be prepared (status "transient", before the command started).
# A call whose command ran is never resubmitted, whatever its exit code.
# usage: tools/gpurun_queue.sh <timeout s> <log file> <command...>
to=$1; log=$2; shift 2
for i in $(seq 1 30); do
  /usr/local/graft/bin/gpurun --timeout "$to" -- "$@" > "$log" 2>&1
  rc=$?
  # the command never started: status "transient" with no run time (busy slots, a box that could
  # not be prepared, back-off)
  notrun=$(python3 -c "import json;d=json.load(open('gpurun_out/.last_call.json'));print(int(d.get('status')=='transient' and not d.get('run_s')))" 2>/dev/null)
  if [ $rc -eq 3 ] || [ "$notrun" = "1" ]; then
    # honour the back-off gpurun asks for ("retry in Ns"), else wait 90 s
    w=$(grep -o "retry in [0-9]*s" "$log" | tail -1 | grep -o "[0-9]*")
    sleep $(( ${w:-80} + 10 )); continue
  fi
  exit $rc
done
exit 3
