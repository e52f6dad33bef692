set -u
mkdir -p gpurun_out/r02n
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread -k "switch or lifecycle or membership or shard or golden" > gpurun_out/r02n/tests.log 2>&1 || { tail -30 gpurun_out/r02n/tests.log; exit 1; }
tail -3 gpurun_out/r02n/tests.log
NFGPU_TRACE_MEMBERSHIP=1 timeout -k 10 300 python tools/membership_bench.py > gpurun_out/r02n/mem_new.json 2>gpurun_out/r02n/mem_new.err && cat gpurun_out/r02n/mem_new.json
