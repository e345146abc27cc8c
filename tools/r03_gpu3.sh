#!/usr/bin/env bash
# Round-3 re-entry GPU pass: suite + smoke + bench (r03_gpu2.sh), then the MALL probe and the config-4 lane statistics.
set -u -o pipefail
bash tools/r03_gpu2.sh && bash tools/r03_mall.sh && bash tools/r03_c4ls.sh
