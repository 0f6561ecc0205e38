# round-3 final, second pass (part A): the full GPU suite, the driver's default N=1 line, its kernel trace
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/r3ga && export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v -s --timeout 600 --timeout-method thread > gpurun_out/r3ga/gputest_full.log 2>&1 || exit 1
timeout -k 10 600 python3 bench.py > gpurun_out/r3ga/bench.json 2> gpurun_out/r3ga/bench.err || exit 2
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r3ga/prof_default -o run -- python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-pmc > gpurun_out/r3ga/default_prof.json 2> gpurun_out/r3ga/default_prof.err || exit 3
