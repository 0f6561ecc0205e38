set -o pipefail
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && O=gpurun_out/r6w && mkdir -p $O
for te in 1 4 1 4; do
timeout -k 10 300 python3 bench.py --steps 200 --warmup 10 --time-every $te > $O/te$te.json 2> $O/te$te.err || exit 1
cat $O/te$te.json >> $O/all.jsonl
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof4 -o run -- python3 bench.py --steps 200 --warmup 10 --time-every 4 > $O/prof4.json 2> $O/prof4.err || exit 2
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof1 -o run -- python3 bench.py --steps 200 --warmup 10 --time-every 1 > $O/prof1.json 2> $O/prof1.err || exit 3
