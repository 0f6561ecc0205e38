set -o pipefail
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && O=gpurun_out/r8d && mkdir -p $O
timeout -k 10 700 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || exit 1
for v in base scan_lanes=3 k5_dyn=0 base scan_lanes=3 k5_dyn=0 base; do
  E=""; [ $v != base ] && E="$v"
  timeout -k 10 300 env PF_DEBUG=$E python3 bench.py --steps 200 --warmup 10 --no-pmc --no-cpu-baseline > $O/b.json 2> $O/b.err || exit 2
  (echo -n "$v "; cat $O/b.json) >> $O/all.txt
done
