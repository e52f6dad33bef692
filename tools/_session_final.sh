set -u
T=${1:-r17o}
mkdir -p gpurun_out/$T
export TMPDIR=/tmp
timeout -k 10 1000 python bench.py --steps 50 --warmup 5 > gpurun_out/$T/bench.log 2> gpurun_out/$T/bench.err
rc=$?
echo "bench rc=$rc"; tail -3 gpurun_out/$T/bench.err
[ $rc -eq 0 ] || exit 1
for c in 1 3 4; do
  B="python bench.py --config $c --steps 20 --warmup 3 --cpu-baseline off --host-calls off --plugin-frame off --other-configs off --adapter-frame off"
  timeout -k 10 -s KILL 300 rocprofv3 --kernel-trace --stats --output-format csv -d $PWD/gpurun_out/$T/stats$c -o run -- $B > gpurun_out/$T/stats$c.log 2>&1
  echo "stats$c rc=$?"
done
SLACKS=8 bash tools/_session_mig.sh $T
