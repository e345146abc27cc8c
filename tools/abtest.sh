#!/usr/bin/env bash
# A/B several builds of librt4.so in one GPU session.
#   build side (here):  tools/abtest.sh build <name>=<git-rev|WORKTREE[:-DFLAG=1 ...]> ...
#   run side (GPU box): tools/abtest.sh run [rounds] [bench args...]
# Variants live in 4d_ray_tracing_amd/lib/variants/<name>.so; bench.py loads one via RT4_LIB.
set -eu
ROOT=$(cd "$(dirname "$0")/.." && pwd)
VDIR=$ROOT/4d_ray_tracing_amd/lib/variants
cmd=${1:-}; shift || true
if [ "$cmd" = build ]; then
  rm -rf "$VDIR"; mkdir -p "$VDIR"
  build_one() {
    local spec=$1 name rev flags tmpo tmp
    name=${spec%%=*}; rev=${spec#*=}
    flags=""
    case "$rev" in WORKTREE:*) flags=${rev#WORKTREE:}; rev=WORKTREE;; esac
    if [ "$rev" = WORKTREE ]; then
      tmpo=$(mktemp -d)
      make -C "$ROOT/4d_ray_tracing_amd/csrc" -s OUT="$tmpo" EXTRA="$flags" "$tmpo/librt4.so" >/dev/null
      cp "$tmpo/librt4.so" "$VDIR/$name.so"
      rm -rf "$tmpo"
    else
      tmp=$(mktemp -d)
      git -C "$ROOT" archive "$rev" 4d_ray_tracing_amd/csrc include | tar -x -C "$tmp"
      make -C "$tmp/4d_ray_tracing_amd/csrc" -s OUT="$tmp/lib" "$tmp/lib/librt4.so" >/dev/null
      cp "$tmp/lib/librt4.so" "$VDIR/$name.so"
      rm -rf "$tmp"
    fi
    echo "built $name ($rev)"
  }
  # the variants build in parallel (one hipcc each; 8 host CPUs)
  pids=()
  for spec in "$@"; do build_one "$spec" & pids+=($!); done
  for p in "${pids[@]}"; do wait "$p" || exit 1; done
elif [ "$cmd" = run ]; then
  rounds=${1:-2}; shift || true
  args=${*:-"--steps 30 --warmup 3 --no-cpu-baseline"}
  for r in $(seq 1 "$rounds"); do
    for so in "$VDIR"/*.so; do
      name=$(basename "$so" .so)
      errf=$(mktemp)
      out=$(RT4_AB_TOLERANT=1 RT4_LIB=$so timeout -k 10 300 python "$ROOT/bench.py" $args 2>"$errf" | tail -1)
      if [ -z "$out" ]; then echo "$name: bench failed:"; tail -5 "$errf"; rm -f "$errf"; continue; fi
      rm -f "$errf"
      python3 - "$name" "$out" <<'PY'
import json, sys
d = json.loads(sys.argv[2])
fr = d.get("roofline", {}).get("frac")
print(f"{sys.argv[1]:>12s}  {d['value']/1e9:8.2f} G int/s  kernel {d['kernel_ms']:.3f} ms  "
      + (f"valu {fr*100:5.2f}%  " if fr else "") + d['config']['scene'])
PY
    done
  done
else
  echo "usage: $0 build name=rev ... | run [rounds] [bench args]"; exit 2
fi
