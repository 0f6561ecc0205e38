# headers loaded before the image staging + pair launches split by image LDS class, vs exp/v/base;
# GPU suite; K5T phase clocks of the new code
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/r3ah && export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v -s --timeout 300 --timeout-method thread -k "not full_size" > gpurun_out/r3ah/gputest.log 2>&1 || exit 1
B="python3 bench.py --workload cfg3 --steps 60 --warmup 5 --no-cpu-baseline --no-pmc"
O=$PWD/exp/v/base/libpokec_fas.so
timeout -k 10 300 $B > gpurun_out/r3ah/cfg3_new.json 2> gpurun_out/r3ah/cfg3_new.err || exit 2
PF_LIB_PATH=$O timeout -k 10 300 $B > gpurun_out/r3ah/cfg3_base.json 2> gpurun_out/r3ah/cfg3_base.err || exit 3
timeout -k 10 300 $B > gpurun_out/r3ah/cfg3_new_b.json 2> gpurun_out/r3ah/cfg3_new_b.err || exit 4
PF_LIB_PATH=$O timeout -k 10 300 $B > gpurun_out/r3ah/cfg3_base_b.json 2> gpurun_out/r3ah/cfg3_base_b.err || exit 5
C="python3 bench.py --workload cfg5 --steps 5 --warmup 2 --contexts 1 --no-cpu-baseline --no-pmc"
timeout -k 10 600 $C > gpurun_out/r3ah/cfg5_c1_new.json 2> gpurun_out/r3ah/cfg5_c1_new.err || exit 6
PF_LIB_PATH=$O timeout -k 10 600 $C > gpurun_out/r3ah/cfg5_c1_base.json 2> gpurun_out/r3ah/cfg5_c1_base.err || exit 7
PF_LIB_PATH=$PWD/exp/v/k5t/libpokec_fas.so timeout -k 10 300 python3 bench.py --workload cfg3 --steps 30 --warmup 3 --no-cpu-baseline --no-pmc > gpurun_out/r3ah/cfg3_k5t.json 2> gpurun_out/r3ah/cfg3_k5t.err || exit 8
