#!/usr/bin/env bash
# Historical (round 3, kept for the logged measurements): RT4_PIPE_MIRROR, the knob this script varies, was
# removed in r03-v35 when the mirror room started pipelining; rebuilding it now gives one binary.
# Config-4 pipelining probe: per-phase lane statistics of the mirror-room tiger kernel,
# frame by frame vs pipelined, from the -DRT4_LANESTATS -DRT4_PIPE_MIRROR=1 build (lib_ls).
set -u -o pipefail
OUT=gpurun_out/r03_c4ls
mkdir -p "$OUT"
export PYTHONUNBUFFERED=1
export RT4_LIB=$PWD/4d_ray_tracing_amd/lib_ls/librt4.so
for mode in fbf pipelined; do
  timeout -k 10 300 python tools/lanestats.py tiger_two_mirrors 16 12 3840 2160 3 $mode > "$OUT/ls_$mode.log" 2>&1 \
    || { echo "lanestats $mode failed"; tail -20 "$OUT/ls_$mode.log"; exit 1; }
  cat "$OUT/ls_$mode.log"
done
for mode in fbf pipelined; do
  timeout -k 10 300 python tools/lanestats.py tiger 16 8 1920 1080 3 $mode > "$OUT/ls_tiger_$mode.log" 2>&1 \
    || { echo "lanestats tiger $mode failed"; tail -20 "$OUT/ls_tiger_$mode.log"; exit 1; }
  cat "$OUT/ls_tiger_$mode.log"
done
echo "c4ls done"
