set -o pipefail
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && O=gpurun_out/r8m && mkdir -p $O
for v in base upload_pad=65536 upload_pad=1048576 base upload_pad=4194304; do
  E=""; [ $v != base ] && E="$v"
  timeout -k 10 300 env PF_DEBUG=$E python3 bench.py --steps 200 --warmup 10 --no-pmc --no-cpu-baseline --no-cfg3 > $O/b.json 2> $O/b.err || exit 2
  (echo -n "$v "; cat $O/b.json) >> $O/all.txt
done
timeout -k 10 300 env PF_DEBUG=upload_pad=1048576 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d $O/tr -o tr -- python3 bench.py --steps 50 --warmup 5 --no-pmc --no-cpu-baseline --no-cfg3 > $O/tr.json 2> $O/tr.err || exit 3
