#!/bin/bash
# Build libadaptive_amd.so variants for A/B runs (tools/ab.sh) into abvar/ (travels to the GPU box).
# usage: bash tools/build_variant.sh <name> <git-rev | WORK> [extra hipcc flags...]
#   WORK = the working tree's sources; a rev = those files as committed at that revision.
set -eu
name=$1; rev=$2; shift 2
ROOT=$(cd "$(dirname "$0")/.." && pwd)
mkdir -p "$ROOT/tools/_build" "$ROOT/abvar"
if [ "$rev" = WORK ]; then  # a snapshot: hipcc reads the sources again for its host pass
  src=$(mktemp -d /tmp/aa_variant.XXXXXX)
  mkdir -p "$src/adaptive_amd" && cp -r "$ROOT/adaptive_amd/csrc" "$src/adaptive_amd/" && cp -r "$ROOT/include" "$src/"
else
  src=$(mktemp -d /tmp/aa_variant.XXXXXX)
  git -C "$ROOT" archive "$rev" adaptive_amd/csrc include | tar -x -C "$src"
fi
/opt/rocm/bin/hipcc -O3 -std=c++17 --offload-arch=gfx950 -fPIC -fvisibility=hidden -ffp-contract=off -Wall \
  -Wno-unused-function -Wno-pass-failed "$@" -I"$src/include" -shared -o "$ROOT/abvar/$name.so" \
  "$src/adaptive_amd/csrc/aa_kernels.hip" "$src/adaptive_amd/csrc/aa_optim.hip"
echo "built abvar/$name.so from $rev $*"
