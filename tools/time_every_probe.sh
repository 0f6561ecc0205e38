cd $GRAFT_REPO_ROOT && O=gpurun_out/r9zzd && mkdir -p $O
for rep in 1 2 3 4; do
  for te in 1 1000; do
    timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 --time-every $te --no-cpu-baseline --no-pmc --no-cfg3 > $O/x.json 2> $O/x.err || exit 1
    (echo -n "s20 te=$te "; tail -1 $O/x.json) >> $O/all.txt
  done
done
for rep in 1 2; do
  for te in 1 1000; do
    timeout -k 10 300 python3 bench.py --steps 200 --warmup 10 --time-every $te --no-cpu-baseline --no-pmc --no-cfg3 > $O/x.json 2> $O/x.err || exit 1
    (echo -n "s200 te=$te "; tail -1 $O/x.json) >> $O/all.txt
  done
done
