#!/bin/bash
# A/B of K5's block hand-out (PF_K5_DYN 0 static / 1 dynamic) on cfg 2 and cfg 4, interleaved:
#   tools/ab_k5dyn.sh <tag>      -> gpurun_out/<tag>/ab_*.json
set -eo pipefail
export TMPDIR=/tmp
T=${1:-r2dyn}
O=gpurun_out/$T; mkdir -p $O
for rep in 1 2; do
  for d in 0 1; do
    PF_K5_DYN=$d timeout -k 10 300 python3 bench.py --steps 200 --warmup 10 --no-cpu-baseline --no-pmc \
        > $O/ab_cfg2_dyn${d}_$rep.json 2> $O/ab_cfg2_dyn${d}_$rep.err
    python3 -c "import json; d=json.load(open('$O/ab_cfg2_dyn${d}_$rep.json')); print('cfg2 dyn=$d rep=$rep', d['value'], round(d['roofline']['avg_launch_ms']*1e3,1), 'us')"
  done
done
for d in 0 1; do
  PF_K5_DYN=$d timeout -k 10 300 python3 bench.py --workload cfg4 --steps 5 --warmup 1 --no-cpu-baseline --no-pmc \
      > $O/ab_cfg4_dyn$d.json 2> $O/ab_cfg4_dyn$d.err
  python3 -c "import json; d=json.load(open('$O/ab_cfg4_dyn$d.json')); print('cfg4 dyn=$d', d['value'])"
done
