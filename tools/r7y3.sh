set -o pipefail
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && O=gpurun_out/r7y3 && mkdir -p $O
for v in old cur old cur old cur old cur; do
  L=""; [ $v = old ] && L="env PF_DEBUG=chunk_pingpong=0"
  timeout -k 10 300 $L python3 bench.py --workload cfg3 --steps 600 --warmup 10 --no-pmc --no-cpu-baseline > $O/cfg3_$v.json 2> $O/cfg3_$v.err || exit 1
  (echo -n "$v "; cat $O/cfg3_$v.json) >> $O/cfg3_all.txt
done
