#!/usr/bin/env bash
# A/B round 12: the claim state packed in one register (r03-v39) against r03-v38; the new bench-shape tests.
set -u -o pipefail
OUT=gpurun_out/r03_ab12
mkdir -p "$OUT"
COMMON="--no-cpu-baseline --no-ops --no-reuse-leg --no-fbf-leg"
bash tools/abtest.sh run 2 --config 5 --steps 32 --warmup 8 $COMMON 2>&1 | tee "$OUT/c5.log" || exit 1
bash tools/abtest.sh run 2 --config 3 --steps 20 --warmup 20 $COMMON 2>&1 | tee "$OUT/c3.log" || exit 1
bash tools/abtest.sh run 1 --config 4 --steps 20 --warmup 3 $COMMON 2>&1 | tee "$OUT/c4.log" || exit 1
bash tools/abtest.sh run 2 --config 2 --steps 20 --warmup 20 $COMMON 2>&1 | tee "$OUT/c2.log" || exit 1
timeout -k 10 600 python -u -m pytest -x -v --timeout 500 --timeout-method thread -m gpu \
  "tests/test_gpu_pipelined.py::test_config4_pipelined_equals_sequential" "tests/test_gpu_pipelined.py::test_lockstep_and_deferral_kernels_1080p" \
  > "$OUT/pytest_new.log" 2>&1 || { echo "pytest failed"; tail -30 "$OUT/pytest_new.log"; exit 1; }
tail -3 "$OUT/pytest_new.log"
echo "ab12 done"
