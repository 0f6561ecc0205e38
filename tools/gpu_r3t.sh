set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/r3t && export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v -s --timeout 300 --timeout-method thread -k "not full_size" > gpurun_out/r3t/gputest.log 2>&1 || exit 1
timeout -k 10 300 python3 bench.py --workload cfg3 --steps 60 --warmup 5 --no-cpu-baseline --no-pmc > gpurun_out/r3t/cfg3.json 2> gpurun_out/r3t/cfg3.err || exit 2
timeout -k 10 300 python3 bench.py --workload cfg3 --steps 60 --warmup 5 --no-cpu-baseline --no-pmc > gpurun_out/r3t/cfg3b.json 2> gpurun_out/r3t/cfg3b.err || exit 2
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r3t/prof_cfg3 -o run -- python3 bench.py --workload cfg3 --steps 30 --warmup 3 --no-cpu-baseline --no-pmc > gpurun_out/r3t/cfg3_prof.json 2> gpurun_out/r3t/cfg3_prof.err || exit 4
timeout -k 10 600 python3 bench.py --workload cfg5 --steps 5 --warmup 2 --contexts 1 --no-cpu-baseline --no-pmc > gpurun_out/r3t/cfg5_c1.json 2> gpurun_out/r3t/cfg5_c1.err || exit 3
timeout -k 10 600 python3 bench.py --workload cfg5 --steps 5 --warmup 2 --no-cpu-baseline --no-pmc > gpurun_out/r3t/cfg5_c3.json 2> gpurun_out/r3t/cfg5_c3.err || exit 5
make -C recommendation-system-pokec_amd clean > /dev/null && make -C recommendation-system-pokec_amd -j16 K5T=1 > gpurun_out/r3t/build_k5t.log 2>&1 || exit 6
timeout -k 10 300 python3 bench.py --workload cfg3 --steps 30 --warmup 3 --no-cpu-baseline --no-pmc > gpurun_out/r3t/cfg3_k5t.json 2> gpurun_out/r3t/cfg3_k5t.err || exit 7
