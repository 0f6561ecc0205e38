#!/bin/bash
# A/B of a K5 profiling knob (an environment variable, 0 vs 1) on cfg 2 (two interleaved
# repetitions of 200 steps) and cfg 4 (one run each):
#   tools/ab_k5.sh <tag> <VAR>      -> gpurun_out/<tag>/ab_<VAR>*.json
set -eo pipefail
export TMPDIR=/tmp
T=$1; V=$2
O=gpurun_out/$T; mkdir -p $O
for rep in 1 2; do
  for d in 0 1; do
    env $V=$d timeout -k 10 300 python3 bench.py --steps 200 --warmup 10 --no-cpu-baseline --no-pmc \
        > $O/ab_${V}_cfg2_${d}_$rep.json 2> $O/ab_${V}_cfg2_${d}_$rep.err
    python3 -c "import json; d=json.load(open('$O/ab_${V}_cfg2_${d}_$rep.json')); print('cfg2 $V=$d rep=$rep', d['value'], round(d['roofline']['avg_launch_ms']*1e3,1), 'us', d['topk_selfcheck'])"
  done
done
for d in 0 1; do
  env $V=$d timeout -k 10 300 python3 bench.py --workload cfg4 --steps 5 --warmup 1 --no-cpu-baseline --no-pmc \
      > $O/ab_${V}_cfg4_$d.json 2> $O/ab_${V}_cfg4_$d.err
  python3 -c "import json; d=json.load(open('$O/ab_${V}_cfg4_$d.json')); print('cfg4 $V=$d', d['value'], d['topk_selfcheck'])"
done
