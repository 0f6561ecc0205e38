set -o pipefail
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && O=gpurun_out/r7g && mkdir -p $O
for v in cur main cur main cur main; do
  L=""; [ $v = main ] && L="env PF_DEBUG=collab_main=1"
  timeout -k 10 300 $L python3 bench.py --workload cfg3 --steps 400 --warmup 10 --no-pmc --no-cpu-baseline > $O/cfg3_$v.json 2> $O/cfg3_$v.err || exit 1
  (echo -n "$v "; cat $O/cfg3_$v.json) >> $O/cfg3_all.txt
done
