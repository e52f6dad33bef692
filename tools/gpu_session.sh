#!/bin/bash
# One GPU session: every GPU step has its own time limit; a crash/abort/timeout stops the
# session (no further GPU work), an ordinary test failure does not.
# usage: tools/gpu_session.sh <tag> [steps...]
#   steps: smoke tests bench prof pmc ablate bench3 bench4 hostprof hbmmix hbmstream pluginbench
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
B="python bench.py --steps 20 --warmup 3 --cpu-baseline off --host-calls off --plugin-frame off ${PMCB:-}"
for step in "$@"; do
  case $step in
    smoke) run smoke 300 python -c "import __graft_entry__ as g; g.smoke()" ;;
    tests) run tests 900 python -u -m pytest tests -m gpu -v --maxfail=5 -p no:cacheprovider \
             --timeout 300 --timeout-method thread ;;
    bench) run bench 600 python bench.py --steps 50 --warmup 5 ;;
    bench0) run bench0 600 python bench.py --config 0 --steps 50 --warmup 5 ;;
    bench3) run bench3 600 python bench.py --config 3 --steps 20 --warmup 3 ${CPUB:---cpu-baseline off} ;;
    bench4) run bench4 600 python bench.py --config 4 --steps 20 --warmup 3 ${CPUB:---cpu-baseline off} ;;
    bench2g) NFGPU_BENCH_TRACE=1 run bench2g 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
               --master-port 29561 bench.py --gpus 2 --steps 20 --warmup 3 --backend gloo --cpu-baseline off \
               --entities 262144 --groups 1024 --migrate 128 ;;
    bench2g1) NFGPU_BENCH_TRACE=1 run bench2g1 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
               --master-port 29562 bench.py --gpus 2 --steps 20 --warmup 3 --backend gloo --cpu-baseline off \
               --entities 262144 --groups 1024 --migrate 128 --migrate-every 1 ;;
    adapter) run adapter 600 python -u -m pytest tests/test_adapter.py tests/test_logic_session.py -m gpu -v -p no:cacheprovider \
             --timeout 300 --timeout-method thread ;;
    abtick) BENCH_ARGS="--other-configs off --plugin-frame off" run abtick 900 tools/ab.sh "$TAG/abtick" ${ABR:-3} $ABLIBS ;;
    abfan) BENCH_ARGS="--config 3 --other-configs off --plugin-frame off" run abfan 900 tools/ab.sh "$TAG/abfan" ${ABR:-2} $ABLIBS ;;
    abrec) BENCH_ARGS="--config 4 --other-configs off --plugin-frame off" run abrec 900 tools/ab.sh "$TAG/abrec" ${ABR:-3} $ABLIBS ;;
    rectests) run rectests 600 python -u -m pytest tests -m gpu -v -p no:cacheprovider --timeout 300 --timeout-method thread -k "record or rec or config4 or golden" ;;
    pfab) BENCH_ARGS="--other-configs off ${PFB:-}" run pfab 900 tools/ab_env.sh "$TAG/pfab" ${PFR:-3} ${PFAB:-NFGPU_TICK_PF=0 NFGPU_TICK_PF=1536 NFGPU_TICK_PF=768 NFGPU_TICK_PF=3072} ;;
    lbab) run lbab 900 tools/ab_env.sh "$TAG/lbab" ${LBR:-4} NFGPU_JIT_LB=1 NFGPU_JIT_LB=0 ;;
    bench2) NFGPU_BENCH_TRACE=1 run bench2 600 python bench.py --gpus 2 --steps 20 --warmup 3 --backend gloo \
               --cpu-baseline off --entities 262144 --groups 1024 --migrate 128 ;;
    ntab) run ntab 900 tools/ab_env.sh "$TAG/ntab" 2 ${NTAB:-NFGPU_JIT_NT=0 NFGPU_JIT_NT=16 NFGPU_JIT_NT=17 NFGPU_JIT_NT=24 NFGPU_JIT_NT=20} ;;
    hostprof) NFGPU_TRACE_EXEC=1 run hostprof 300 python tools/host_calls_profile.py ;;
    hbmmix) run hbmmix 120 tools/_bin/hbm_mix ;;
    hbmstream) run hbmstream 240 tools/_bin/hbm_stream ;;
    plugintests) run plugintests 600 python -u -m pytest tests -m gpu -v -p no:cacheprovider --timeout 300 --timeout-method thread \
                     -k "plugin or functor or adapter or logic_session or shard" ;;
    pluginab) run pluginab 900 python tools/plugin_frame_ab.py --rounds ${PABR:-2} ${PAB:-NFGPU_PLUGIN_THREADS=0 NFGPU_PLUGIN_THREADS=4 NFGPU_PLUGIN_THREADS=8} ;;
    repeat) run repeat 900 tools/repeat_test.sh "$TAG/repeat" ${RR:-3} "${RK:-plugin_shard_replay}" ;;
    repeatpack) LIBDIR=ab/pack run repeatpack 900 tools/repeat_test.sh "$TAG/repeatpack" ${RR:-3} "${RK:-plugin_shard_replay}" ;;
    repeatbase) LIBDIR=ab/base run repeatbase 900 tools/repeat_test.sh "$TAG/repeatbase" ${RR:-3} "${RK:-plugin_shard_replay}" ;;
    pluginbench) run pluginbench 600 python bench.py --steps 20 --warmup 3 --cpu-baseline off --host-calls off ;;
    membership) NFGPU_TRACE_MEMBERSHIP=1 run membership 300 python tools/membership_bench.py ;;
    selfmigcpp) run selfmigcpp 300 python bench.py --self-migrate --shard cpp --steps 24 --warmup 8 --cpu-baseline off \
               --host-calls off --plugin-frame off --other-configs off ;;
    selfmig) NFGPU_BENCH_TRACE=1 NFGPU_TRACE_EXEC=1 NFGPU_TRACE_MEMBERSHIP=1 run selfmig 300 python bench.py --self-migrate \
               --steps 24 --warmup 8 --cpu-baseline off --host-calls off ;;
    ablate) run ablate 600 python tools/ablate.py --variants ${ABL:-0,8,4} ;;
    prof)  run prof 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof" -o run -- \
             python bench.py --steps 50 --warmup 5 --cpu-baseline off --host-calls off --plugin-frame off ;;
    prof4) run prof4 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof4" -o run -- \
             python bench.py --config 4 --steps 20 --warmup 3 --cpu-baseline off --host-calls off --plugin-frame off ;;
    pmc)
      run calib_fetch 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$OUT/calib_fetch" -o run -- \
        tools/_bin/pmc_calib
      run calib_write 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$OUT/calib_write" -o run -- \
        tools/_bin/pmc_calib
      run pmc_fetch 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$OUT/pmc_fetch" -o run -- $B
      run pmc_write 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$OUT/pmc_write" -o run -- $B
      run pmc_sq 300 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY \
        SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR TCC_HIT_sum TCC_MISS_sum GRBM_GUI_ACTIVE \
        --output-format csv -d "$OUT/pmc_sq" -o run -- $B
      ALG="$OUT/bench.log"; [ -f "$ALG" ] || ALG=""
      run pmc_summary 60 python tools/pmc_summary.py --calib "$OUT/calib_fetch" "$OUT/calib_write" \
        --bench "$OUT/pmc_fetch" "$OUT/pmc_write" --sq "$OUT/pmc_sq" ${ALG:+--alg "$ALG"} \
        --out "$OUT/pmc_traffic.json" ;;
    abifloor) run abifloor 120 tools/_bin/ref_abi_floor ;;
    *) echo "unknown step $step" ;;
  esac
done
echo "session done"
