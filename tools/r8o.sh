set -o pipefail
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && O=gpurun_out/r8o && mkdir -p $O
timeout -k 10 300 env PF_DEBUG=lane_zc=1 python -u -m pytest tests/test_gpu_parity.py -x -q -m gpu --timeout 120 --timeout-method thread -k "scan_lanes or profile_sampling or sharded_single" > $O/tests.log 2>&1 || exit 1
for v in base lane_zc=1 lane_zc=2 base lane_zc=1; do
  E=""; [ $v != base ] && E="$v"
  timeout -k 10 300 env PF_DEBUG=$E python3 bench.py --steps 200 --warmup 10 --no-pmc --no-cpu-baseline --no-cfg3 > $O/b.json 2> $O/b.err || exit 2
  (echo -n "$v "; cat $O/b.json) >> $O/all.txt
done
