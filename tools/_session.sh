set -u
T=${1:-r17c}
mkdir -p gpurun_out/$T
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -v --timeout 300 --timeout-method thread -p no:cacheprovider -m gpu tests/test_logic_session.py -k "gpu_plugin_matches and 78" > gpurun_out/$T/tests.log 2>&1
echo "tests rc=$?"
tail -4 gpurun_out/$T/tests.log
timeout -k 10 600 tools/prof_config0.sh $T/c0
echo "prof_config0 rc=$?"
timeout -k 10 700 tools/prof_adapter.sh 2 $T/npc
echo "prof_adapter rc=$?"
