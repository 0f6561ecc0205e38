#!/bin/bash
# Round profile on the GPU box (run through gpurun from the repo root):
#   tools/profile_round.sh <tag> [scan kernel: postings|stream]
# 1. rocprofv3 --pmc FETCH_SIZE pass over a short bench (its own run, no tracing)
#    -> HBM bytes per scan-kernel launch (x2 gfx950 correction, MI355X_MICROARCH.md HBM)
# 2. rocprofv3 --kernel-trace --stats over the default bench command
# 3. the default bench line (with the CPU baseline), reading the traffic from step 1
# Everything lands in gpurun_out/<tag>/; copy the summaries into profiles/ afterwards.
set -eo pipefail
export TMPDIR=/tmp
T=${1:-r1}
SK=${2:-postings}
K=fas_post_kernel; [ "$SK" = stream ] && K=fas_scan_kernel
O=gpurun_out/$T
mkdir -p $O
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex $K -T --output-format csv \
    -d $O/pmc -o run -- python3 bench.py --steps 20 --warmup 3 --no-cpu-baseline --scan-kernel $SK > $O/pmc.log 2>&1
python3 tools/pmc_summary.py $O/pmc workload_from=$O/pmc.log kernel=$K > $O/pmc_traffic.json
python3 - $O/pmc_traffic.json <<'PY'
import json, sys, os
p = "profiles/pmc_traffic.json"
d = json.load(open(p)) if os.path.exists(p) else {}
d.update(json.load(open(sys.argv[1])))
json.dump(d, open(p, "w"), indent=1)
PY
timeout -k 10 300 rocprofv3 --kernel-trace --stats -T --output-format csv -d $O/trace -o run \
    -- python3 bench.py --steps 50 --warmup 5 --no-cpu-baseline --scan-kernel $SK > $O/trace.log 2>&1
timeout -k 10 400 python3 bench.py --scan-kernel $SK > $O/bench.json 2> $O/bench.err
cp profiles/pmc_traffic.json $O/pmc_traffic_all.json
cat $O/bench.json
