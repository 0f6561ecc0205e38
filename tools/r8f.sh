set -o pipefail
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && O=gpurun_out/r8f && mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q -m gpu --timeout 120 --timeout-method thread -k "scan_lanes or profile_sampling or async" > $O/tests.log 2>&1 || exit 1
for v in base base base; do
  E=""; [ $v != base ] && E="$v"
  timeout -k 10 300 env PF_DEBUG=$E python3 bench.py --steps 200 --warmup 10 --no-pmc --no-cpu-baseline > $O/b.json 2> $O/b.err || exit 2
  (echo -n "$v "; cat $O/b.json) >> $O/all.txt
done
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/tr -o tr -- python3 bench.py --steps 50 --warmup 5 --no-pmc --no-cpu-baseline > $O/tr.json 2> $O/tr.err || exit 3
