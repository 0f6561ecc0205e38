set -o pipefail
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && O=gpurun_out/r7y4 && mkdir -p $O
for v in old cur old cur old cur; do
  L=""; [ $v = old ] && L="env PF_DEBUG=chunk_pingpong=0"
  timeout -k 10 300 $L python3 bench.py --steps 5 --warmup 2 --no-pmc --no-cpu-baseline > $O/b_$v.json 2> $O/b_$v.err || exit 1
  (echo -n "$v "; cat $O/b_$v.json) >> $O/all.txt
done
