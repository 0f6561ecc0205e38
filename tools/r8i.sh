set -o pipefail
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && O=gpurun_out/r8i && mkdir -p $O
for v in host_prof=1; do
  timeout -k 10 300 env PF_DEBUG=$v python3 bench.py --steps 200 --warmup 10 --no-pmc --no-cpu-baseline > $O/b.json 2> $O/b_$v.err || exit 2
  (echo -n "$v "; cat $O/b.json) >> $O/all.txt
done
