#!/bin/bash
# Interleaved A/B timing of environment settings (e.g. NFGPU_JIT=0 vs 1) on one box: each round
# runs bench.py once per setting, in separate processes, under its own time limit.
#   tools/ab_env.sh <tag> <rounds> "ENV=a" "ENV=b" ...
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=$1; R=$2; shift 2
OUT=gpurun_out/$TAG; mkdir -p "$OUT"
for r in $(seq 1 "$R"); do
  i=0
  for e in "$@"; do
    i=$((i+1))
    env $e timeout -k 5 180 python bench.py --steps 50 --warmup 5 --cpu-baseline off --host-calls off --plugin-frame off ${BENCH_ARGS:-} \
      > "$OUT/v${i}_$r.log" 2>&1 || { echo "fail $e"; tail -3 "$OUT/v${i}_$r.log"; exit 1; }
    python -c "
import json; d=json.loads(open('$OUT/v${i}_$r.log').read().strip().splitlines()[-1])
print('$e', $r, round(d['ms_per_step']*1000,1), {k: round(v['avg_us'],1) for k,v in d['kernels'].items()})"
  done
done
