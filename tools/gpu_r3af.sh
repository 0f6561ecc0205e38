# K4' with the collaborative top-k fused in (K8 skips those jobs) vs exp/v/nofuse; GPU subset
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/r3af && export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v -s --timeout 300 --timeout-method thread -k "not full_size" > gpurun_out/r3af/gputest.log 2>&1 || exit 1
B="python3 bench.py --workload cfg3 --steps 60 --warmup 5 --no-cpu-baseline --no-pmc --async-depth 2"
N=$PWD/exp/v/nofuse/libpokec_fas.so
timeout -k 10 300 $B > gpurun_out/r3af/cfg3_fuse.json 2> gpurun_out/r3af/cfg3_fuse.err || exit 2
PF_LIB_PATH=$N timeout -k 10 300 $B > gpurun_out/r3af/cfg3_nofuse.json 2> gpurun_out/r3af/cfg3_nofuse.err || exit 3
timeout -k 10 300 $B > gpurun_out/r3af/cfg3_fuse_b.json 2> gpurun_out/r3af/cfg3_fuse_b.err || exit 4
PF_LIB_PATH=$N timeout -k 10 300 $B > gpurun_out/r3af/cfg3_nofuse_b.json 2> gpurun_out/r3af/cfg3_nofuse_b.err || exit 5
C="python3 bench.py --workload cfg5 --steps 5 --warmup 2 --contexts 1 --no-cpu-baseline --no-pmc"
timeout -k 10 600 $C > gpurun_out/r3af/cfg5_c1_fuse.json 2> gpurun_out/r3af/cfg5_c1_fuse.err || exit 6
PF_LIB_PATH=$N timeout -k 10 600 $C > gpurun_out/r3af/cfg5_c1_nofuse.json 2> gpurun_out/r3af/cfg5_c1_nofuse.err || exit 7
