set -u
mkdir -p gpurun_out/r16f
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -v --timeout 300 --timeout-method thread -p no:cacheprovider -m gpu tests/test_tutorial3.py tests/test_logic_session.py tests/test_adapter.py tests/test_shard_cpp.py > gpurun_out/r16f/tests.log 2>&1
echo "tests rc=$?"
tail -4 gpurun_out/r16f/tests.log
timeout -k 10 1000 python bench.py --steps 50 --warmup 5 > gpurun_out/r16f/bench.log 2> gpurun_out/r16f/bench.err
echo "bench rc=$?"
tail -3 gpurun_out/r16f/bench.err
