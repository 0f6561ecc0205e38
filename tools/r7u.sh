# cfg4 with every query the same user (perfect list sharing in L2) vs the seeded stream: bounds what a
# query-tiled batch could save
set -o pipefail
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && O=gpurun_out/r7u && mkdir -p $O
timeout -k 10 300 python3 bench.py --workload cfg4 --steps 3 --warmup 1 --no-pmc --no-cpu-baseline > $O/cfg4.json 2> $O/cfg4.err || exit 1
timeout -k 10 300 python3 bench.py --workload cfg4 --steps 3 --warmup 1 --no-pmc --no-cpu-baseline --same-query > $O/cfg4_same.json 2> $O/cfg4_same.err || exit 2
timeout -k 10 300 python3 bench.py --steps 50 --warmup 5 --no-pmc --no-cpu-baseline --no-cfg3 --same-query > $O/cfg2_same.json 2> $O/cfg2_same.err || exit 3
