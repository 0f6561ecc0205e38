# final pass with kHitCap 20: full GPU suite, the default line, its rocprof summary, cfg3 / cfg5 lines,
# and the record-stream scan (K1, which spills 64 B per lane at cap 20) against exp/v/hc16
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/r3aj && export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v -s --timeout 600 --timeout-method thread > gpurun_out/r3aj/gputest_full.log 2>&1 || exit 1
timeout -k 10 600 python3 bench.py > gpurun_out/r3aj/bench.json 2> gpurun_out/r3aj/bench.err || exit 2
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r3aj/prof_default -o run -- python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-pmc > gpurun_out/r3aj/default_prof.json 2> gpurun_out/r3aj/default_prof.err || exit 3
timeout -k 10 600 python3 bench.py --workload cfg3 > gpurun_out/r3aj/cfg3.json 2> gpurun_out/r3aj/cfg3.err || exit 4
S="python3 bench.py --scan-kernel stream --steps 30 --warmup 5 --no-cpu-baseline --no-pmc"
timeout -k 10 300 $S > gpurun_out/r3aj/k1_hc20.json 2> gpurun_out/r3aj/k1_hc20.err || exit 5
PF_LIB_PATH=$PWD/exp/v/hc16/libpokec_fas.so timeout -k 10 300 $S > gpurun_out/r3aj/k1_hc16.json 2> gpurun_out/r3aj/k1_hc16.err || exit 6
