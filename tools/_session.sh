set -u
T=${1:-r17q}
mkdir -p gpurun_out/$T
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -p no:cacheprovider -m gpu tests/test_gpu_parity.py tests/test_shard_cpp.py > gpurun_out/$T/tests.log 2>&1
rc=$?
echo "tests rc=$rc"; tail -2 gpurun_out/$T/tests.log
[ $rc -eq 0 ] || exit 1
SLACKS=8 bash tools/_session_mig.sh $T
timeout -k 10 1000 python bench.py --steps 50 --warmup 5 > gpurun_out/$T/bench.log 2> gpurun_out/$T/bench.err
echo "bench rc=$?"; tail -2 gpurun_out/$T/bench.err
