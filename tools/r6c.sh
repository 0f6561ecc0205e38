# round-5 A/B call: slice kernel (PF_DEBUG k5_slice=1) variants, ticket ordering
set -o pipefail
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp
PF_DEBUG=k5_slice=1 bash tools/gpu_round.sh r6c quick quickv:r4 k5t quick4 || exit 1
bash tools/gpu_round.sh r6c_base quick quickv:relaxed quick4 || exit 2
bash tools/gpu_round.sh r6c_base cfg3v:relaxed || exit 3
timeout -k 10 600 python3 bench.py --workload cfg3 --steps 30 --warmup 5 --no-cpu-baseline --no-pmc > gpurun_out/r6c_base/cfg3.json 2> gpurun_out/r6c_base/cfg3.err || exit 4
timeout -k 10 600 python3 bench.py --workload cfg4 --steps 3 --warmup 1 --no-cpu-baseline --no-pmc --solo-shards 8 > gpurun_out/r6c_base/cfg4_solo.json 2> gpurun_out/r6c_base/cfg4_solo.err || exit 5
