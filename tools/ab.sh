#!/bin/bash
# Interleaved A/B timing of libnfgpu builds on config[1] (or BENCH_ARGS): each round runs bench.py
# once per library, in separate processes, under its own time limit.
#   tools/ab.sh <tag> <rounds> lib1.so lib2.so ...
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=$1; R=$2; shift 2
OUT=gpurun_out/$TAG; mkdir -p "$OUT"
for r in $(seq 1 "$R"); do
  for lib in "$@"; do
    n=$(basename "$lib" .so)
    NFGPU_LIB=$PWD/$lib timeout -k 5 120 python bench.py --steps 50 --warmup 5 --cpu-baseline off --host-calls off ${BENCH_ARGS:-} \
      > "$OUT/${n}_$r.log" 2>&1 || { echo "fail $n"; tail -3 "$OUT/${n}_$r.log"; exit 1; }
    python -c "
import json; d=json.loads(open('$OUT/${n}_$r.log').read().strip().splitlines()[-1])
print('$n', $r, round(d['ms_per_step']*1000,1), {k: round(v['avg_us'],1) for k,v in d['kernels'].items()})"
  done
done
