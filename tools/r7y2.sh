set -o pipefail
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && O=gpurun_out/r7y2 && mkdir -p $O
for v in cur old cur old cur old; do
  L=""; [ $v = old ] && L="env PF_DEBUG=chunk_pingpong=0"
  timeout -k 10 300 $L python3 bench.py --workload cfg3 --steps 400 --warmup 10 --no-pmc --no-cpu-baseline > $O/cfg3_$v.json 2> $O/cfg3_$v.err || exit 1
  (echo -n "$v "; cat $O/cfg3_$v.json) >> $O/cfg3_all.txt
done
for v in cur old cur old; do
  L=""; [ $v = old ] && L="env PF_DEBUG=chunk_pingpong=0"
  timeout -k 10 400 $L python3 bench.py --workload cfg5 --no-pmc --no-cpu-baseline > $O/cfg5_$v.json 2> $O/cfg5_$v.err || exit 2
  (echo -n "$v "; cat $O/cfg5_$v.json) >> $O/cfg5_all.txt
done
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 600 --timeout-method thread > $O/gputest.log 2>&1 || exit 3
