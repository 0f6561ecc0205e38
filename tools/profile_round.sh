#!/bin/bash
# Round profile on the GPU box (run through gpurun from the repo root):
#   tools/profile_round.sh <tag>
# 1. rocprofv3 --pmc FETCH_SIZE pass over a short bench (its own run, no tracing)
#    -> HBM bytes per fas_scan_kernel launch (x2 gfx950 correction, MI355X_MICROARCH.md HBM)
# 2. rocprofv3 --kernel-trace --stats over the default bench command
# 3. the default bench line (with the CPU baseline), reading the traffic from step 1
# Everything lands in gpurun_out/<tag>/; copy the summaries into profiles/ afterwards.
set -eo pipefail
export TMPDIR=/tmp
T=${1:-r1}
O=gpurun_out/$T
mkdir -p $O
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex fas_scan -T --output-format csv \
    -d $O/pmc -o run -- python3 bench.py --steps 20 --warmup 3 --no-cpu-baseline > $O/pmc.log 2>&1
python3 tools/pmc_summary.py $O/pmc workload_from=$O/pmc.log > $O/pmc_traffic.json
cp $O/pmc_traffic.json profiles/pmc_traffic.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats -T --output-format csv -d $O/trace -o run \
    -- python3 bench.py --steps 50 --warmup 5 --no-cpu-baseline > $O/trace.log 2>&1
timeout -k 10 400 python3 bench.py > $O/bench.json 2> $O/bench.err
cat $O/bench.json
