#!/bin/bash
# Build a libnfgpu variant for A/B timing (tools/ab.sh) into ab/<name>.so, from a git revision
# (its tracked sources, in a scratch copy) or from the working tree ("-"), with extra hipcc flags.
#   tools/ab_build.sh <name> <rev|-> [hipcc flags...]
set -eu
cd "$(dirname "$0")/.."
NAME=$1; REV=$2; shift 2
ROOT=$PWD
SRC=$ROOT
if [ "$REV" != "-" ]; then
  SRC=$(mktemp -d)
  trap 'rm -rf "$SRC"' EXIT
  git archive "$REV" __graft_entry__.py include noahgameframe_amd | tar -x -C "$SRC"
fi
mkdir -p ab
(cd "$SRC" && python -c "import __graft_entry__ as g; g.jit_source()")
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -fPIC -shared -Wall -Wno-unused-result \
  "$@" -o "ab/$NAME.so" "$SRC/noahgameframe_amd/csrc/nfgpu_host.hip" -lhiprtc
echo "built ab/$NAME.so from $REV"
