# one stream per job workspace slot (consecutive calls overlap on the device): correctness subset,
# cfg 3 / cfg 5 lines, host stage clocks, a kernel trace
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/r3y && export TMPDIR=/tmp
timeout -k 10 700 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v -s --timeout 300 --timeout-method thread -k "collab or recommenders or set_adj or pipelined or async or contexts or variants or digests or holdout or facade" > gpurun_out/r3y/gputest_sub.log 2>&1 || exit 1
B="python3 bench.py --workload cfg3 --steps 60 --warmup 5 --no-cpu-baseline --no-pmc"
timeout -k 10 300 $B > gpurun_out/r3y/cfg3.json 2> gpurun_out/r3y/cfg3.err || exit 2
timeout -k 10 300 $B > gpurun_out/r3y/cfg3_b.json 2> gpurun_out/r3y/cfg3_b.err || exit 3
PF_DEBUG=host_prof=1 timeout -k 10 300 $B > gpurun_out/r3y/cfg3_hp.json 2> gpurun_out/r3y/cfg3_hp.err || exit 4
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r3y/prof_cfg3 -o run -- $B > gpurun_out/r3y/cfg3_prof.json 2> gpurun_out/r3y/cfg3_prof.err || exit 5
timeout -k 10 600 python3 bench.py --workload cfg5 --steps 5 --warmup 2 --contexts 1 --no-cpu-baseline --no-pmc > gpurun_out/r3y/cfg5_c1.json 2> gpurun_out/r3y/cfg5_c1.err || exit 6
timeout -k 10 600 python3 bench.py --workload cfg5 --steps 5 --warmup 2 --no-cpu-baseline --no-pmc > gpurun_out/r3y/cfg5_c3.json 2> gpurun_out/r3y/cfg5_c3.err || exit 7
