#!/usr/bin/env bash
# gpurun with retries ONLY for infrastructure-side failures where nothing ran (box not prepared, no free slot).
# A command that ran and failed is never re-run. Usage: tools/gpu.sh <timeout-seconds> '<command>'
T=$1
shift
for attempt in 1 2 3 4 5 6; do
  out=$(/usr/local/graft/bin/gpurun --timeout "$T" -- "$@" 2>&1)
  rc=$?
  if echo "$out" | grep -qE "status=transient|no free box|stopped responding while being prepared|are busy" || [ $rc -eq 3 ]; then
    echo "[gpu.sh] attempt $attempt: infrastructure not ready, waiting" >&2
    sleep $((30 * attempt))
    continue
  fi
  echo "$out"
  exit $rc
done
echo "$out"
exit 3
