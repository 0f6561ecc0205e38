set -o pipefail
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && O=gpurun_out/r7h && mkdir -p $O
for v in cur main cur main; do
  L=""; [ $v = main ] && L="env PF_DEBUG=collab_main=1"
  timeout -k 10 400 $L python3 bench.py --workload cfg5 --no-pmc --no-cpu-baseline > $O/cfg5_$v.json 2> $O/cfg5_$v.err || exit 1
  (echo -n "$v "; cat $O/cfg5_$v.json) >> $O/cfg5_all.txt
done
