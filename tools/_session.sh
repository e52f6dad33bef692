set -u
T=${1:-r17t}
mkdir -p gpurun_out/$T
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread -p no:cacheprovider -m gpu \
  tests/test_gpu_boundary.py tests/test_logic_session.py \
  "tests/test_gpu_parity.py::test_gpu_matches_oracle" -k "validation or logic_session or const_guards or set_ops" \
  > gpurun_out/$T/tests.log 2>&1
rc=$?
echo "tests rc=$rc"; tail -2 gpurun_out/$T/tests.log
exit $rc
