# round-3 final (part B): cfg3 / cfg4 / cfg5 lines (CPU baseline + PMC pass each), cfg5 at one
# context with host stage clocks, an N=2 rehearsal over gloo on one GPU
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/r3fb && export TMPDIR=/tmp
timeout -k 10 600 python3 bench.py --workload cfg3 > gpurun_out/r3fb/cfg3.json 2> gpurun_out/r3fb/cfg3.err || exit 1
timeout -k 10 600 python3 bench.py --workload cfg4 > gpurun_out/r3fb/cfg4.json 2> gpurun_out/r3fb/cfg4.err || exit 2
timeout -k 10 900 python3 bench.py --workload cfg5 > gpurun_out/r3fb/cfg5.json 2> gpurun_out/r3fb/cfg5.err || exit 3
PF_DEBUG=host_prof=1 timeout -k 10 600 python3 bench.py --workload cfg5 --steps 5 --warmup 2 --contexts 1 --no-cpu-baseline --no-pmc > gpurun_out/r3fb/cfg5_c1.json 2> gpurun_out/r3fb/cfg5_c1.err || exit 4
timeout -k 10 600 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 2 --dist-backend gloo --steps 5 --warmup 2 --no-pmc > gpurun_out/r3fb/rehearsal_n2_gloo.json 2> gpurun_out/r3fb/rehearsal_n2_gloo.err || exit 5
