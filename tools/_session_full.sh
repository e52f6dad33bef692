set -u
T=${1:-r17m}
mkdir -p gpurun_out/$T
export TMPDIR=/tmp
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/$T/smoke.log 2>&1
echo "smoke rc=$?"; tail -2 gpurun_out/$T/smoke.log
timeout -k 10 1000 python -u -m pytest -v --timeout 300 --timeout-method thread -p no:cacheprovider -m gpu tests/ > gpurun_out/$T/gpu_tests.log 2>&1
rc=$?
echo "gpu tests rc=$rc"
tail -4 gpurun_out/$T/gpu_tests.log
