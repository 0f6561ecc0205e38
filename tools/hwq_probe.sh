# probe: hardware queues per process (GPU_MAX_HW_QUEUES) x scan lanes x one-query workgroups, cfg2
cd $GRAFT_REPO_ROOT && O=gpurun_out/$1 && mkdir -p $O && shift
run() { # tag hwq pfdebug
  timeout -k 10 300 env GPU_MAX_HW_QUEUES=$2 PF_DEBUG=$3 python3 bench.py --steps 200 --warmup 10 --no-cpu-baseline --no-pmc --no-cfg3 > $O/$1.json 2> $O/$1.err || exit 1
  (echo -n "$1 hwq=$2 $3 "; tail -1 $O/$1.json) >> $O/all.txt
}
for rep in 1 2; do
  for spec in "$@"; do
    IFS=/ read -r h d <<< "$spec"
    run "q${h}_${d//[=,]/_}_$rep" $h $d
  done
done
