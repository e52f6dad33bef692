#!/bin/bash
# One GPU session: every GPU step has its own time limit; a crash/abort/timeout stops the
# session (no further GPU work), an ordinary test failure does not.
# usage: tools/gpu_session.sh <tag> [steps...]   steps: smoke tests bench prof pmc
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=${1:-r01}; shift
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
run() {  # run <name> <seconds> <cmd...>
  local name=$1 secs=$2; shift 2
  echo "=== $name: $*" | tee -a "$OUT/session.log"
  timeout -k 10 "$secs" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc" | tee -a "$OUT/session.log"
  tail -n 5 "$OUT/$name.log"
  case $rc in
    0|1) return 0 ;;          # pass / test failures: keep going
    *) echo "fatal rc=$rc in $name, stopping" | tee -a "$OUT/session.log"; exit $rc ;;
  esac
}
for step in "$@"; do
  case $step in
    smoke) run smoke 300 python -c "import __graft_entry__ as g; g.smoke()" ;;
    tests) run tests 900 python -m pytest tests -m gpu -q --maxfail=5 -p no:cacheprovider ;;
    bench) run bench 600 python bench.py --steps 50 --warmup 5 ;;
    prof)  run prof 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof" -o run -- \
             python bench.py --steps 50 --warmup 5 --cpu-baseline off ;;
    pmc)   run pmc_fetch 600 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$OUT/pmc_fetch" -o run -- \
             python bench.py --steps 20 --warmup 3 --cpu-baseline off &&
           run pmc_write 600 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$OUT/pmc_write" -o run -- \
             python bench.py --steps 20 --warmup 3 --cpu-baseline off ;;
    *) echo "unknown step $step" ;;
  esac
done
echo "session done"
