set -u
T=${1:-r17s}
mkdir -p gpurun_out/$T
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -p no:cacheprovider -m gpu tests/test_shard_cpp.py tests/test_adapter.py > gpurun_out/$T/tests.log 2>&1
rc=$?
echo "tests rc=$rc"; tail -2 gpurun_out/$T/tests.log
[ $rc -eq 0 ] || exit 1
SLACKS="8 8" bash tools/_session_mig.sh $T
grep "shard begin" gpurun_out/$T/selfmig_s8.err | tail -4
