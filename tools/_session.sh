set -u
T=${1:-r18b}
mkdir -p gpurun_out/$T
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread -p no:cacheprovider -m gpu \
  tests/test_gpu_boundary.py tests/test_gpu_parity.py tests/test_adapter.py \
  -k "boundary or lookups or folding or object_index or (matches_oracle and k_tick] ) or golden or adapter_session or schedule" \
  > gpurun_out/$T/tests.log 2>&1
rc=$?
echo "tests rc=$rc"; tail -2 gpurun_out/$T/tests.log
[ $rc -eq 0 ] || exit 1
timeout -k 10 400 python -u tools/host_calls_profile.py --frames 30 > gpurun_out/$T/hc.log 2> gpurun_out/$T/hc.err
rc=$?
echo "hc rc=$rc"; tail -1 gpurun_out/$T/hc.log
exit $rc
