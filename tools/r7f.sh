set -o pipefail
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && O=gpurun_out/r7f && mkdir -p $O
for v in cur main cur main; do
  L=""; [ $v = main ] && L="env PF_DEBUG=collab_main=1"
  timeout -k 10 300 $L python3 bench.py --workload cfg3 --steps 50 --warmup 5 --no-pmc > $O/cfg3_$v.json 2> $O/cfg3_$v.err || exit 1
  (echo -n "$v "; cat $O/cfg3_$v.json) >> $O/cfg3_all.txt
done
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 600 --timeout-method thread > $O/gputest.log 2>&1 || exit 2
