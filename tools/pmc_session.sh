#!/bin/bash
# PMC traffic of the frame kernels for configs 1, 3, 4 (one calibration, then per config: the bench line
# for the algorithmic bytes, FETCH_SIZE and WRITE_SIZE in separate passes, an SQ/TCC pass) and a
# rocprofv3 --kernel-trace --stats run per config; every GPU step under its own time limit, the session
# stops at the first failure.   tools/pmc_session.sh <tag> [configs...]
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=$1; shift
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
step() {  # step <name> <seconds> <cmd...>
  local name=$1 secs=$2; shift 2
  echo "=== $name" | tee -a "$OUT/session.log"
  timeout -k 10 -s KILL "$secs" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc" | tee -a "$OUT/session.log"
  [ $rc -eq 0 ] || { tail -5 "$OUT/$name.log"; exit $rc; }
}
step calib_fetch 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$OUT/calib_fetch" -o run -- tools/_bin/pmc_calib
step calib_write 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$OUT/calib_write" -o run -- tools/_bin/pmc_calib
for c in "${@:-1 3 4}"; do
  B="python bench.py --config $c --steps 20 --warmup 3 --cpu-baseline off --host-calls off --plugin-frame off --other-configs off --adapter-frame off"
  step bench$c 300 $B
  step pmc_fetch$c 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$OUT/pmc_fetch$c" -o run -- $B
  step pmc_write$c 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$OUT/pmc_write$c" -o run -- $B
  step pmc_sq$c 300 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY \
    SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR TCC_HIT_sum TCC_MISS_sum GRBM_GUI_ACTIVE \
    --output-format csv -d "$OUT/pmc_sq$c" -o run -- $B
  step stats$c 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/stats$c" -o run -- $B
  python tools/pmc_summary.py --calib "$OUT/calib_fetch" "$OUT/calib_write" --bench "$OUT/pmc_fetch$c" "$OUT/pmc_write$c" \
    --sq "$OUT/pmc_sq$c" --alg "$OUT/bench$c.log" --out "$OUT/pmc_config$c.json" > /dev/null
done
echo "session done"
