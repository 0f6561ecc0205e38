set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/r3u && export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v -s --timeout 300 --timeout-method thread -k "not full_size" > gpurun_out/r3u/gputest.log 2>&1 || exit 1
timeout -k 10 300 python3 bench.py --workload cfg3 --steps 60 --warmup 5 --no-cpu-baseline --no-pmc > gpurun_out/r3u/cfg3.json 2> gpurun_out/r3u/cfg3.err || exit 2
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r3u/prof_cfg3 -o run -- python3 bench.py --workload cfg3 --steps 30 --warmup 3 --no-cpu-baseline --no-pmc > gpurun_out/r3u/cfg3_prof.json 2> gpurun_out/r3u/cfg3_prof.err || exit 4
make -C recommendation-system-pokec_amd clean > /dev/null && make -C recommendation-system-pokec_amd -j16 K5T=1 > gpurun_out/r3u/build_k5t.log 2>&1 || exit 6
timeout -k 10 300 python3 bench.py --workload cfg3 --steps 30 --warmup 3 --no-cpu-baseline --no-pmc > gpurun_out/r3u/cfg3_k5t.json 2> gpurun_out/r3u/cfg3_k5t.err || exit 7
