#!/bin/bash
# Repeats one -m gpu test selection R times (a determinism check), optionally against another
# libnfgpu.so directory (LIBDIR: put in front of the in-tree library for the C++ test clients).
#   tools/repeat_test.sh <tag> <rounds> <-k expression>
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=$1; R=$2; K=$3
OUT=gpurun_out/$TAG; mkdir -p "$OUT"
for r in $(seq 1 "$R"); do
  LD_LIBRARY_PATH=${LIBDIR:+$PWD/$LIBDIR:}${LD_LIBRARY_PATH:-} timeout -k 10 300 python -u -m pytest tests -m gpu -q \
    -p no:cacheprovider --timeout 240 --timeout-method thread -k "$K" > "$OUT/run_$r.log" 2>&1
  rc=$?
  echo "round $r rc=$rc $(tail -1 "$OUT/run_$r.log")"
  [ $rc -le 1 ] || exit $rc
done
