set -u
mkdir -p gpurun_out/r03d
for v in 16777216 33554432; do
NFGPU_ABLATE=$v timeout -k 10 300 python -c "
from noahgameframe_amd import workload
from tests.parity import run_gpu, run_oracle, compare_runs
for seed, ppg in ((1, 16), (2, 24), (3, 40)):
    w = workload.make_world(n_obj=4000, n_scenes=2, groups_per_scene=8, players_per_group=ppg, n_ticks=6, seed=seed, ext_frac=0.05)
    compare_runs(run_gpu(w), run_oracle(w))
print('fan window parity ok $v')
" || exit 1
done
BENCH_ARGS="--config 4 --steps 20 --warmup 3" bash tools/ab_env.sh r03d4 2 NFGPU_ABLATE=0 NFGPU_ABLATE=16777216 NFGPU_ABLATE=33554432
BENCH_ARGS="--config 3 --steps 10 --warmup 2" bash tools/ab_env.sh r03d3 2 NFGPU_ABLATE=0 NFGPU_ABLATE=16777216 NFGPU_ABLATE=33554432
