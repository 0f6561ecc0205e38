# three asynchronous calls in flight (three workspace slots) vs two: async tests, cfg 3 A/B, timeline
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/r3ae && export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v -s --timeout 300 --timeout-method thread -k "async or contexts or collab" > gpurun_out/r3ae/gputest_sub.log 2>&1 || exit 1
B="python3 bench.py --workload cfg3 --steps 60 --warmup 5 --no-cpu-baseline --no-pmc"
timeout -k 10 300 $B > gpurun_out/r3ae/cfg3_d3.json 2> gpurun_out/r3ae/cfg3_d3.err || exit 2
timeout -k 10 300 $B --async-depth 2 > gpurun_out/r3ae/cfg3_d2.json 2> gpurun_out/r3ae/cfg3_d2.err || exit 3
timeout -k 10 300 $B > gpurun_out/r3ae/cfg3_d3_b.json 2> gpurun_out/r3ae/cfg3_d3_b.err || exit 4
timeout -k 10 300 $B --async-depth 2 > gpurun_out/r3ae/cfg3_d2_b.json 2> gpurun_out/r3ae/cfg3_d2_b.err || exit 5
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r3ae/prof_cfg3 -o run -- $B > gpurun_out/r3ae/cfg3_prof.json 2> gpurun_out/r3ae/cfg3_prof.err || exit 6
