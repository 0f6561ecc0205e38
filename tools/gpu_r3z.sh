# K3 gathers forked onto an aux stream beside the K6 images: correctness subset, cfg 3 / cfg 5 lines, trace
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/r3z && export TMPDIR=/tmp
timeout -k 10 700 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v -s --timeout 300 --timeout-method thread -k "collab or recommenders or set_adj or pipelined or async or contexts or variants or digests or holdout or facade or gathers" > gpurun_out/r3z/gputest_sub.log 2>&1 || exit 1
B="python3 bench.py --workload cfg3 --steps 60 --warmup 5 --no-cpu-baseline --no-pmc"
timeout -k 10 300 $B > gpurun_out/r3z/cfg3.json 2> gpurun_out/r3z/cfg3.err || exit 2
timeout -k 10 300 $B > gpurun_out/r3z/cfg3_b.json 2> gpurun_out/r3z/cfg3_b.err || exit 3
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r3z/prof_cfg3 -o run -- $B > gpurun_out/r3z/cfg3_prof.json 2> gpurun_out/r3z/cfg3_prof.err || exit 4
timeout -k 10 600 python3 bench.py --workload cfg5 --steps 5 --warmup 2 --contexts 1 --no-cpu-baseline --no-pmc > gpurun_out/r3z/cfg5_c1.json 2> gpurun_out/r3z/cfg5_c1.err || exit 5
timeout -k 10 600 python3 bench.py --workload cfg5 --steps 5 --warmup 2 --no-cpu-baseline --no-pmc > gpurun_out/r3z/cfg5_c3.json 2> gpurun_out/r3z/cfg5_c3.err || exit 6
