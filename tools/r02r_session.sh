set -u
mkdir -p gpurun_out/r02r
NFGPU_ABLATE=8388608 timeout -k 10 300 python -c "
from noahgameframe_amd import workload
from tests.parity import run_gpu, run_oracle, compare_runs
for seed in (1, 2):
    w = workload.make_world(n_obj=3000, n_scenes=2, groups_per_scene=4, players_per_group=6, records=True, rec_rows=64, n_ticks=8, seed=seed)
    compare_runs(run_gpu(w), run_oracle(w))
print('recvec parity ok')
" || exit 1
BENCH_ARGS="--config 4 --steps 20 --warmup 3" bash tools/ab_env.sh r02r 3 NFGPU_ABLATE=0 NFGPU_ABLATE=8388608
