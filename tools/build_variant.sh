#!/bin/bash
# Build libadaptive_amd.so variants for A/B runs (tools/ab.sh) into tools/_build/.
# usage: bash tools/build_variant.sh <name> <git-rev | WORK> [extra hipcc flags...]
#   WORK = the working tree's sources; a rev = those files as committed at that revision.
set -eu
name=$1; rev=$2; shift 2
ROOT=$(cd "$(dirname "$0")/.." && pwd)
mkdir -p "$ROOT/tools/_build"
if [ "$rev" = WORK ]; then  # a snapshot: hipcc reads the sources again for its host pass
  src=$(mktemp -d /tmp/aa_variant.XXXXXX)
  mkdir -p "$src/adaptive_amd" && cp -r "$ROOT/adaptive_amd/csrc" "$src/adaptive_amd/" && cp -r "$ROOT/include" "$src/"
else
  src=$(mktemp -d /tmp/aa_variant.XXXXXX)
  git -C "$ROOT" archive "$rev" adaptive_amd/csrc include | tar -x -C "$src"
fi
/opt/rocm/bin/hipcc -O3 -std=c++17 --offload-arch=gfx950 -fPIC -fvisibility=hidden -ffp-contract=off -Wall \
  -Wno-unused-function -Wno-pass-failed "$@" -I"$src/include" -shared -o "$ROOT/tools/_build/$name.so" \
  "$src/adaptive_amd/csrc/aa_kernels.hip"
echo "built tools/_build/$name.so from $rev $*"
