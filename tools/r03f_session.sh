set -u
mkdir -p gpurun_out/r03f
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread -k "oracle or golden or config1 or config3" > gpurun_out/r03f/tests.log 2>&1 || { tail -30 gpurun_out/r03f/tests.log; exit 1; }
tail -2 gpurun_out/r03f/tests.log
bash tools/ab.sh r03f 3 noahgameframe_amd/_ab/lib_base.so noahgameframe_amd/_ab/lib_nobar.so
