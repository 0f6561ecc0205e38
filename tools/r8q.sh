set -o pipefail
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && O=gpurun_out/r8q && mkdir -p $O
for v in base k5_batch_blocks=32 k5_batch_blocks=8 base k5_batch_blocks=32 k5_batch_blocks=24 base; do
  E=""; [ $v != base ] && E="$v"
  timeout -k 10 300 env PF_DEBUG=$E python3 bench.py --workload cfg4 --steps 4 --warmup 1 --no-pmc --no-cpu-baseline > $O/b.json 2> $O/b.err || exit 2
  (echo -n "$v "; cat $O/b.json) >> $O/all.txt
done
