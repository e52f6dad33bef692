set -u
mkdir -p gpurun_out/r02y
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread -k "records or config4" > gpurun_out/r02y/tests.log 2>&1 || { tail -30 gpurun_out/r02y/tests.log; exit 1; }
tail -2 gpurun_out/r02y/tests.log
BENCH_ARGS="--config 4 --steps 20 --warmup 3" bash tools/ab.sh r02y 3 noahgameframe_amd/_ab/lib_ballot.so noahgameframe_amd/_ab/lib_readlane.so
