# round-3 final, second pass (part B): cfg3 / cfg4 / cfg5 lines (CPU baseline + PMC pass each), cfg5 at
# one context against the previous commit's library in alternating order, an N=2 gloo rehearsal
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/r3gb && export TMPDIR=/tmp
timeout -k 10 900 python3 bench.py --workload cfg5 > gpurun_out/r3gb/cfg5.json 2> gpurun_out/r3gb/cfg5.err || exit 1
C="python3 bench.py --workload cfg5 --steps 5 --warmup 2 --contexts 1 --no-cpu-baseline --no-pmc"
O=$PWD/exp/v/base/libpokec_fas.so
PF_LIB_PATH=$O timeout -k 10 600 $C > gpurun_out/r3gb/cfg5_c1_base.json 2> gpurun_out/r3gb/cfg5_c1_base.err || exit 2
timeout -k 10 600 $C > gpurun_out/r3gb/cfg5_c1_new.json 2> gpurun_out/r3gb/cfg5_c1_new.err || exit 3
PF_LIB_PATH=$O timeout -k 10 600 $C > gpurun_out/r3gb/cfg5_c1_base_b.json 2> gpurun_out/r3gb/cfg5_c1_base_b.err || exit 4
timeout -k 10 600 $C > gpurun_out/r3gb/cfg5_c1_new_b.json 2> gpurun_out/r3gb/cfg5_c1_new_b.err || exit 5
timeout -k 10 600 python3 bench.py --workload cfg3 > gpurun_out/r3gb/cfg3.json 2> gpurun_out/r3gb/cfg3.err || exit 6
timeout -k 10 600 python3 bench.py --workload cfg4 > gpurun_out/r3gb/cfg4.json 2> gpurun_out/r3gb/cfg4.err || exit 7
timeout -k 10 600 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 2 --dist-backend gloo --steps 5 --warmup 2 --no-pmc > gpurun_out/r3gb/rehearsal_n2_gloo.json 2> gpurun_out/r3gb/rehearsal_n2_gloo.err || exit 8
