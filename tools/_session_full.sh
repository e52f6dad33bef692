set -u
T=${1:-r17h}
mkdir -p gpurun_out/$T
export TMPDIR=/tmp
timeout -k 10 960 python -u -m pytest -x -v --timeout 300 --timeout-method thread -p no:cacheprovider -m gpu tests/ > gpurun_out/$T/gpu_tests.log 2>&1
rc=$?
echo "gpu tests rc=$rc"
tail -4 gpurun_out/$T/gpu_tests.log
[ $rc -eq 0 ] || exit 1
SLACKS=8 bash tools/_session_mig.sh $T
