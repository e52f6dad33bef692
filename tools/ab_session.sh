#!/bin/bash
# One A/B session: GPU parity of the in-tree library, then interleaved timing of library builds
# on config[1] and (optionally) config[3] / config[4].
#   tools/ab_session.sh <tag> <rounds> "<configs>" lib1.so lib2.so ...
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=$1; R=$2; CFGS=$3; shift 3
mkdir -p gpurun_out/$TAG
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread \
  > gpurun_out/$TAG/tests.log 2>&1; rc=$?
tail -3 gpurun_out/$TAG/tests.log
[ $rc -le 1 ] || exit $rc
for c in $CFGS; do
  envs=()
  for lib in "$@"; do envs+=("NFGPU_LIB=$lib"); done
  BENCH_ARGS="--config $c ${BENCH_EXTRA:-}" bash tools/ab_env.sh "$TAG/c$c" "$R" "${envs[@]}" || exit 1
done
