#!/bin/bash
# Submit one gpurun call from this container, resubmitting only while gpurun reports that no box
# or slot was free (nothing ran, nothing charged); any call that ran is final.
# Usage: tools/gpu_submit.sh LOG TIMEOUT 'command'
LOG=$1; T=$2; CMD=$3
for attempt in 1 2 3 4 5 6 7 8 9 10 11 12; do
    timeout $((T + 1500)) /usr/local/graft/bin/gpurun --timeout "$T" -- "$CMD" > "$LOG" 2>&1
    rc=$?
    if grep -q "status=transient" "$LOG" && grep -q "no free box\|nothing was charged\|stopped responding while being prepared\|backing off\|taken away by the GPU service" "$LOG" \
       && ! grep -q "status=ok" "$LOG"; then
        sleep 120
        continue
    fi
    break
done
echo "gpu_submit rc=$rc attempts=$attempt" >> "$LOG"
