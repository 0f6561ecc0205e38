# round-5: asynchronous cfg-5 driver calls (tests, then cfg 5 async vs --eval-sync)
set -o pipefail
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out/r6h
bash tools/gpu_round.sh r6h "tests:async or driver or holdout or pipelined" || exit 1
Q="--no-cpu-baseline --no-pmc"
timeout -k 10 900 python3 bench.py --workload cfg5 --steps 5 --warmup 2 $Q > gpurun_out/r6h/cfg5_async.json 2> gpurun_out/r6h/cfg5_async.err || exit 2
timeout -k 10 900 python3 bench.py --workload cfg5 --steps 5 --warmup 2 $Q --eval-sync > gpurun_out/r6h/cfg5_sync.json 2> gpurun_out/r6h/cfg5_sync.err || exit 3
timeout -k 10 900 python3 bench.py --workload cfg5 --steps 10 --warmup 2 $Q > gpurun_out/r6h/cfg5_async10.json 2> gpurun_out/r6h/cfg5_async10.err || exit 4
timeout -k 10 700 bash tools/pmc_passes.sh r6h_k1p fas_pairs --workload cfg3 --steps 10 --warmup 2 || exit 5
