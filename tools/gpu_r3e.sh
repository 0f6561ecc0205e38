set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/r3e && export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v -s --timeout 300 --timeout-method thread -k "not full_size" > gpurun_out/r3e/gputest.log 2>&1 || exit 1
timeout -k 10 300 python3 bench.py --workload cfg3 --steps 60 --warmup 5 --no-cpu-baseline --no-pmc > gpurun_out/r3e/cfg3.json 2> gpurun_out/r3e/cfg3.err || exit 2
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r3e/prof_cfg3 -o run -- python3 bench.py --workload cfg3 --steps 30 --warmup 3 --no-cpu-baseline --no-pmc > gpurun_out/r3e/cfg3_prof.json 2> gpurun_out/r3e/cfg3_prof.err || exit 4
