#!/bin/bash
# Round profile on the GPU box (run through gpurun from the repo root):
#   tools/profile_round.sh <tag> [scan kernel: postings|stream]
# 1. FETCH_SIZE calibration (tools/fetch_calib under rocprofv3 --pmc) -> the gfx950 factor
#    for K5's load widths, written to profiles/fetch_calib_r2.json (bench.py reads it)
# 2. rocprofv3 --kernel-trace --stats over the bench command (no CPU baseline, no PMC pass)
# 3. the default bench line: CPU baseline + its own rocprofv3 --pmc FETCH_SIZE pass + the run
# Everything lands in gpurun_out/<tag>/; copy the summaries into profiles/ afterwards.
set -eo pipefail
export TMPDIR=/tmp
T=${1:-r2}
SK=${2:-postings}
O=gpurun_out/$T
mkdir -p $O
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -T --output-format csv -d $O/calib -o run \
    -- tools/fetch_calib > $O/fetch_calib.out 2> $O/fetch_calib.err
python3 tools/fetch_calib.py $O/calib $O/fetch_calib.out > $O/fetch_calib.json
cp $O/fetch_calib.json profiles/fetch_calib_r2.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats -T --output-format csv -d $O/trace -o run \
    -- python3 bench.py --steps 50 --warmup 5 --no-cpu-baseline --no-pmc --scan-kernel $SK > $O/trace.log 2>&1
timeout -k 10 600 python3 bench.py --scan-kernel $SK > $O/bench.json 2> $O/bench.err
cat $O/bench.json
