#!/usr/bin/env bash
# One bench line per BASELINE config / scene on one GPU (run on the GPU box from the repo root).
# Config 4 and 5 are 8-GPU configs: one GPU's share (3840 x 270 = 1/8 of 4K) is measured here.
set -u
B="timeout -k 10 300 python bench.py --no-cpu-baseline"
run() { echo "== $*"; $B "$@" 2>/dev/null | tail -1 || return 1; }
run --scene sphere
run --scene hypercube                                   # BASELINE config 3
run --scene room
run --scene tiger
run --scene cylinder4d
run --scene tiger_two_mirrors --width 3840 --height 270 --spp 64 --bounces 12 --steps 5 --warmup 1   # config 4, 1/8
run --scene all_primitives --width 3840 --height 270 --spp 16 --bounces 8 --format f16 --steps 10    # config 5 frame, 1/8
run --scene sphere --format f16
run --scene sphere --format rgba8
