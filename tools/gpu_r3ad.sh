# cfg 3 async-region timeline with the early gathers (kernel trace)
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/r3ad && export TMPDIR=/tmp
B="python3 bench.py --workload cfg3 --steps 60 --warmup 5 --no-cpu-baseline --no-pmc"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r3ad/prof_cfg3 -o run -- $B > gpurun_out/r3ad/cfg3_prof.json 2> gpurun_out/r3ad/cfg3_prof.err || exit 1
PF_DEBUG=host_prof=1 timeout -k 10 300 $B > gpurun_out/r3ad/cfg3_hp.json 2> gpurun_out/r3ad/cfg3_hp.err || exit 2
