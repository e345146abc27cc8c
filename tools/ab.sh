#!/usr/bin/env bash
# The one A/B and profiling driver (replaces round 3's one-off tools/r03_*.sh scripts).
#
#   here (CPU, builds):
#     tools/ab.sh build name=<git-rev|WORKTREE>[:-DFLAG=1 ...] ...
#         builds each variant of librt4.so into 4d_ray_tracing_amd/lib/variants/<name>.so
#   on the GPU box (gpurun), from the repo root:
#     tools/ab.sh run <tag> <rounds> "<configs>" <leg> ...
#         leg = <label>[=<variant>][:<bench arg>+<bench arg>...]; the variant defaults to the label,
#         "tree" is the in-tree build. Prints one line per (round, config, leg): kernel ms per frame and
#         G int/s, interleaved round by round (noise: compare legs of the same round and box).
#     tools/ab.sh prof <tag> "<configs>" [variant]
#         rocprofv3 kernel trace + PMC passes at the bench's launch shape (tools/profile_configs.sh),
#         summarised per config into gpurun_out/prof_<tag>_config<c>/summary.json
#     tools/ab.sh check <tag>
#         the driver's round-end commands: pytest -m gpu, smoke(), the default bench line
# Every step runs under its own time limit and the script stops at the first failure.
set -u -o pipefail
ROOT=$(cd "$(dirname "$0")/.." && pwd)
VDIR=$ROOT/4d_ray_tracing_amd/lib/variants
COMMON="--no-cpu-baseline --no-ops --no-reuse-leg --no-fbf-leg --no-sections-leg --no-steady-leg"
export PYTHONUNBUFFERED=1

steps_of() {  # the bench shape per BASELINE config: as many warmup frames as timed ones (clock ramp)
  case $1 in
    4) echo "--steps 2 --warmup 1" ;;
    5) echo "--steps 32 --warmup 8" ;;
    *) echo "--steps 20 --warmup 20" ;;
  esac
}

cmd=${1:-}
shift || true
case "$cmd" in
build)
  rm -rf "$VDIR"
  mkdir -p "$VDIR"
  build_one() {
    local spec=$1 name rev flags tmp
    name=${spec%%=*}
    rev=${spec#*=}
    flags=""
    case "$rev" in WORKTREE:*) flags=${rev#WORKTREE:}; rev=WORKTREE ;; esac
    tmp=$(mktemp -d)
    if [ "$rev" = WORKTREE ]; then
      make -C "$ROOT/4d_ray_tracing_amd/csrc" -s OUT="$tmp" EXTRA="$flags" "$tmp/librt4.so" > /dev/null || return 1
      cp "$tmp/librt4.so" "$VDIR/$name.so"
    else
      git -C "$ROOT" archive "$rev" 4d_ray_tracing_amd/csrc include | tar -x -C "$tmp"
      make -C "$tmp/4d_ray_tracing_amd/csrc" -s OUT="$tmp/lib" "$tmp/lib/librt4.so" > /dev/null || return 1
      cp "$tmp/lib/librt4.so" "$VDIR/$name.so"
    fi
    rm -rf "$tmp"
    echo "built $name ($rev $flags)"
  }
  pids=()
  for spec in "$@"; do
    build_one "$spec" &
    pids+=($!)
  done
  for p in "${pids[@]}"; do wait "$p" || exit 1; done
  ;;
run)
  TAG=$1 R=$2 CONFIGS=$3
  shift 3
  OUT=$ROOT/gpurun_out/ab_$TAG
  mkdir -p "$OUT"
  for r in $(seq 1 "$R"); do
    for c in $CONFIGS; do
      for leg in "$@"; do
        label=${leg%%[=:]*}
        rest=${leg#"$label"}
        variant=$label
        args=""
        case "$rest" in =*) variant=${rest#=}; variant=${variant%%:*} ;; esac
        case "$rest" in *:*) args=${rest#*:}; args=${args//+/ } ;; esac
        lib=""
        [ "$variant" != tree ] && lib=$VDIR/$variant.so
        log=$OUT/${label}_c${c}_r$r.log
        # shellcheck disable=SC2046
        RT4_AB_TOLERANT=1 RT4_LIB=${lib:-$ROOT/4d_ray_tracing_amd/lib/librt4.so} timeout -k 10 600 \
          python "$ROOT/bench.py" --config "$c" $(steps_of "$c") $COMMON $args > "$log" 2>&1 \
          || { echo "$label config $c: bench failed"; tail -5 "$log"; exit 1; }
        python3 - "$label" "$c" "$r" "$(tail -1 "$log")" << 'PY' | tee -a "$OUT/ab.log"
import json, sys
d = json.loads(sys.argv[4])
print(f"r{sys.argv[3]} config {sys.argv[2]} {sys.argv[1]:>14s}  {d['kernel_ms']:8.4f} ms  {d['value'] / 1e9:7.2f} G int/s")
PY
      done
    done
  done
  echo "ab $TAG done"
  ;;
prof)
  TAG=$1 CONFIGS=$2 VARIANT=${3:-tree}
  if [ "$VARIANT" != tree ]; then export RT4_LIB=$VDIR/$VARIANT.so RT4_AB_TOLERANT=1; fi
  bash "$ROOT/tools/profile_configs.sh" "$TAG" $CONFIGS || exit 1
  ;;
check)
  TAG=$1
  OUT=$ROOT/gpurun_out/check_$TAG
  mkdir -p "$OUT"
  timeout -k 10 900 python -u -m pytest "$ROOT/tests" -m gpu -x -v --timeout 600 --timeout-method thread \
    --durations=15 > "$OUT/pytest_gpu.log" 2>&1 || { echo "pytest failed"; tail -40 "$OUT/pytest_gpu.log"; exit 1; }
  tail -3 "$OUT/pytest_gpu.log"
  timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1 \
    || { echo "smoke failed"; tail -20 "$OUT/smoke.log"; exit 1; }
  tail -2 "$OUT/smoke.log"
  timeout -k 10 300 python3 "$ROOT/bench.py" --gpus 1 --steps 20 --warmup 5 > "$OUT/bench.log" 2>&1 \
    || { echo "bench failed"; tail -20 "$OUT/bench.log"; exit 1; }
  tail -1 "$OUT/bench.log" | cut -c1-400
  ;;
*)
  sed -n '2,20p' "$0"
  exit 2
  ;;
esac
