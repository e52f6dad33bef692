set -u
BENCH_ARGS="--config 4 --steps 20 --warmup 3" bash tools/ab.sh r02z4 2 noahgameframe_amd/_ab/lib_ballot.so noahgameframe_amd/_ab/lib_scan16.so
bash tools/ab.sh r02z1 2 noahgameframe_amd/_ab/lib_ballot.so noahgameframe_amd/_ab/lib_scan16.so
