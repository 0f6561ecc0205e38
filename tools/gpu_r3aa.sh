# resident query images (built at open) + K3 beside K6: GPU suite, cfg 3 / cfg 5 lines, trace, open stages
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/r3aa && export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v -s --timeout 300 --timeout-method thread -k "not full_size" > gpurun_out/r3aa/gputest.log 2>&1 || exit 1
B="python3 bench.py --workload cfg3 --steps 60 --warmup 5 --no-cpu-baseline --no-pmc"
PF_DEBUG=host_prof=1 timeout -k 10 300 $B > gpurun_out/r3aa/cfg3.json 2> gpurun_out/r3aa/cfg3.err || exit 2
timeout -k 10 300 $B > gpurun_out/r3aa/cfg3_b.json 2> gpurun_out/r3aa/cfg3_b.err || exit 3
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r3aa/prof_cfg3 -o run -- $B > gpurun_out/r3aa/cfg3_prof.json 2> gpurun_out/r3aa/cfg3_prof.err || exit 4
timeout -k 10 600 python3 bench.py --workload cfg5 --steps 5 --warmup 2 --contexts 1 --no-cpu-baseline --no-pmc > gpurun_out/r3aa/cfg5_c1.json 2> gpurun_out/r3aa/cfg5_c1.err || exit 5
timeout -k 10 600 python3 bench.py --workload cfg5 --steps 5 --warmup 2 --no-cpu-baseline --no-pmc > gpurun_out/r3aa/cfg5_c3.json 2> gpurun_out/r3aa/cfg5_c3.err || exit 6
