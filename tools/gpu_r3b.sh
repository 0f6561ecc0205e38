set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/r3b && export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests -m gpu -x -v -s --timeout 300 --timeout-method thread -k "any_token_ids or pipelined or two_contexts or async" > gpurun_out/r3b/gputest_rest.log 2>&1 || exit 1
timeout -k 10 600 python3 bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r3b/bench.json 2> gpurun_out/r3b/bench.err || exit 2
export PF_DEBUG=host_prof=1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r3b/prof_cfg3c1 -o run -- python3 bench.py --workload cfg3 --contexts 1 --steps 30 --warmup 3 --no-cpu-baseline --no-pmc > gpurun_out/r3b/cfg3c1.json 2> gpurun_out/r3b/cfg3c1.err || exit 3
