# re-entry check of HEAD: GPU suite (without the full-size tests), the default line, cfg 3 and cfg 5 at one context
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/r3v && export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v -s --timeout 300 --timeout-method thread -k "not full_size" > gpurun_out/r3v/gputest.log 2>&1 || exit 1
timeout -k 10 300 python3 bench.py --steps 50 --warmup 5 --no-pmc > gpurun_out/r3v/default.json 2> gpurun_out/r3v/default.err || exit 2
timeout -k 10 300 python3 bench.py --workload cfg3 --steps 60 --warmup 5 --no-cpu-baseline --no-pmc > gpurun_out/r3v/cfg3.json 2> gpurun_out/r3v/cfg3.err || exit 3
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r3v/prof_cfg3 -o run -- python3 bench.py --workload cfg3 --steps 30 --warmup 3 --no-cpu-baseline --no-pmc > gpurun_out/r3v/cfg3_prof.json 2> gpurun_out/r3v/cfg3_prof.err || exit 4
