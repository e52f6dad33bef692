set -u
mkdir -p gpurun_out/r02q
NFGPU_LIB=$PWD/noahgameframe_amd/_ab/lib_rt16.so timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread -k "records and not touch" > gpurun_out/r02q/tests_rt16.log 2>&1 || { tail -30 gpurun_out/r02q/tests_rt16.log; exit 1; }
tail -2 gpurun_out/r02q/tests_rt16.log
BENCH_ARGS="--config 4 --steps 20 --warmup 3" bash tools/ab.sh r02q 2 noahgameframe_amd/_ab/lib_rt64.so noahgameframe_amd/_ab/lib_rt32.so noahgameframe_amd/_ab/lib_rt16.so
