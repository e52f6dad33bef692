set -u
T=${1:-r17d}
mkdir -p gpurun_out/$T
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread -p no:cacheprovider -m gpu tests/test_gpu_parity.py > gpurun_out/$T/parity.log 2>&1
rc=$?
echo "parity rc=$rc"
tail -4 gpurun_out/$T/parity.log
[ $rc -eq 0 ] || exit 1
BENCH_ARGS="--config 4 --other-configs off --adapter-frame off" timeout -k 10 600 tools/ab_env.sh $T/ab 3 "NFGPU_REC_FLAT=0" "NFGPU_REC_FLAT=1" > gpurun_out/$T/ab.txt 2>&1
echo "ab rc=$?"
cat gpurun_out/$T/ab.txt
