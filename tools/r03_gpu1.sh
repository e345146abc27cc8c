#!/usr/bin/env bash
# Historical (round 3, kept for the logged measurements): RT4_PIPE_MIRROR, the knob this script varies, was
# removed in r03-v35 when the mirror room started pipelining; rebuilding it now gives one binary.
# Round-3 first GPU pass: the new parity tests (bench-shape pipelined frames, C++ RCCL bands path,
# unpermute), the default bench line, and bench-shape profiles of every config, plus config 4 pipelined
# (the RT4_PIPE_MIRROR=1 variant library) for the pipelined-vs-frame-by-frame counter diff.
set -u -o pipefail
OUT=gpurun_out/r03_gpu${GPU_TAG:-1}
mkdir -p "$OUT"
export PYTHONUNBUFFERED=1
timeout -k 10 900 python -u -m pytest -x -v --timeout 600 --timeout-method thread \
  tests/test_gpu_pipelined.py tests/test_gpu_shard.py "tests/test_gpu_configs.py::test_bench_call_1080p_bitwise" \
  tests/test_gpu_native_math.py -s \
  > "$OUT/pytest_new.log" 2>&1 || { echo "pytest failed"; tail -40 "$OUT/pytest_new.log"; exit 1; }
tail -3 "$OUT/pytest_new.log"
timeout -k 10 300 python bench.py > "$OUT/bench_default.log" 2>&1 || { echo "bench failed"; tail -20 "$OUT/bench_default.log"; exit 1; }
tail -1 "$OUT/bench_default.log" | cut -c1-400
bash tools/profile_configs.sh r03v33 2 3 4 5 || exit 1
RT4_LIB=$PWD/4d_ray_tracing_amd/lib_pipemirror/librt4.so bash tools/profile_configs.sh r03v33pm 4 || exit 1
echo "gpu1 done"
