# K1u union walk: collaborative GPU tests, cfg 3 with / without friend groups (same binary), GPU suite
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/r3w && export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v -s --timeout 300 --timeout-method thread -k "collab or recommenders or big_collab or set_adj or pipelined or async or variants" > gpurun_out/r3w/gputest_collab.log 2>&1 || exit 1
timeout -k 10 300 python3 bench.py --workload cfg3 --steps 60 --warmup 5 --no-cpu-baseline --no-pmc > gpurun_out/r3w/cfg3.json 2> gpurun_out/r3w/cfg3.err || exit 2
PF_DEBUG=union=0 timeout -k 10 300 python3 bench.py --workload cfg3 --steps 60 --warmup 5 --no-cpu-baseline --no-pmc > gpurun_out/r3w/cfg3_nounion.json 2> gpurun_out/r3w/cfg3_nounion.err || exit 3
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r3w/prof_cfg3 -o run -- python3 bench.py --workload cfg3 --steps 30 --warmup 3 --no-cpu-baseline --no-pmc > gpurun_out/r3w/cfg3_prof.json 2> gpurun_out/r3w/cfg3_prof.err || exit 4
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v -s --timeout 300 --timeout-method thread -k "not full_size" > gpurun_out/r3w/gputest.log 2>&1 || exit 5
