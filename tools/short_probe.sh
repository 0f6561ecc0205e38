# probe: the driver's short cfg-2 line (--steps 20 --warmup 5) under several PF_DEBUG / queue settings, R reps each
# usage: tools/short_probe.sh TAG R SPEC...   (SPEC = hwq/pfdebug, '-' for none)
cd $GRAFT_REPO_ROOT && O=gpurun_out/$1 && mkdir -p $O && R=$2 && shift 2
for rep in $(seq $R); do
  for spec in "$@"; do
    IFS=/ read -r h d <<< "$spec"
    [ "$d" = "-" ] && d=""
    timeout -k 10 300 env PF_DEBUG=$d python3 bench.py --steps 20 --warmup 5 --hw-queues $h --no-cpu-baseline --no-pmc --no-cfg3 > $O/x.json 2> $O/x.err || exit 1
    (echo -n "$spec "; tail -1 $O/x.json) >> $O/all.txt
  done
done
