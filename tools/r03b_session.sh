set -u
mkdir -p gpurun_out/r03b
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread -k "records or config4" > gpurun_out/r03b/tests.log 2>&1 || { tail -30 gpurun_out/r03b/tests.log; exit 1; }
tail -2 gpurun_out/r03b/tests.log
BENCH_ARGS="--config 4 --steps 20 --warmup 3" bash tools/ab.sh r03b 3 noahgameframe_amd/_ab/lib_ballot.so noahgameframe_amd/_ab/lib_sbytes.so
for f in gpurun_out/r03b/lib_*_1.log; do tail -1 $f | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$f', d['kernels']['k_records']['alg_bytes_per_launch'])"; done
