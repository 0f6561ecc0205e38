#!/bin/bash
# The other BASELINE configurations' bench lines on the GPU box (run through gpurun from the
# repo root), each with its CPU baseline and its own rocprofv3 --pmc FETCH_SIZE pass:
#   tools/round_lines.sh <tag>      -> gpurun_out/<tag>/cfg{3,4,5}.json (+ .err)
# cfg 2 (the metric's configuration) is tools/profile_round.sh.
set -eo pipefail
export TMPDIR=/tmp
T=${1:-r2}
O=gpurun_out/$T
mkdir -p $O
timeout -k 10 600 python3 bench.py --workload cfg3 --steps 60 --warmup 6 > $O/cfg3.json 2> $O/cfg3.err
timeout -k 10 600 python3 bench.py --workload cfg4 --steps 10 --warmup 2 > $O/cfg4.json 2> $O/cfg4.err
timeout -k 10 900 python3 bench.py --workload cfg5 --steps 3 --warmup 1 > $O/cfg5.json 2> $O/cfg5.err
for w in cfg3 cfg4 cfg5; do
  python3 -c "import json; d=json.load(open('$O/$w.json')); r=d['roofline']; print('$w', d['value'], d['unit'], 'ms/step', round(d['ms_per_step'],3), 'frac', r['frac'], 'dram_frac', r['dram_frac'], 'x cpu', d.get('speedup_vs_cpu'))"
done
