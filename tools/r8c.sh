set -o pipefail
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && O=gpurun_out/r8c && mkdir -p $O
for v in k5_dyn=1 base k5_dyn=1,k5_wgs=992 k5_dyn=1,k5_wgs=896 k5_dyn=1,k5_xcd=0 k5_dyn=1 base k5_dyn=1,k5_wgs=1008; do
  E=""; [ $v != base ] && E="$v"
  timeout -k 10 300 env PF_DEBUG=$E python3 bench.py --steps 200 --warmup 10 --no-pmc --no-cpu-baseline > $O/b.json 2> $O/b.err || exit 1
  (echo -n "$v "; cat $O/b.json) >> $O/all.txt
done
