#!/bin/bash
# k_records instruction mix / icache counters for one library + env (config[4], one pass each)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=$1; shift
OUT=gpurun_out/$TAG; mkdir -p "$OUT"
export TMPDIR=/tmp
B="python bench.py --config 4 --other-configs off --steps 10 --warmup 2 --cpu-baseline off --host-calls off --plugin-frame off"
timeout -s KILL 120 rocprofv3 --pmc SQC_ICACHE_HITS SQC_ICACHE_MISSES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_INSTS_SMEM SQ_WAVES \
  --output-format csv -d "$OUT/pmc_i" -o run -- $B > "$OUT/pmc_i.log" 2>&1
