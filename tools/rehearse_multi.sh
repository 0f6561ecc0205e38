#!/bin/bash
# bench.py's N > 1 path with all ranks on the box's one GPU (--dist-backend gloo: collectives
# through host memory), as a correctness rehearsal of the driver's 8-GPU runs:
#   tools/rehearse_multi.sh <tag> <N> [workload]     -> gpurun_out/<tag>/n<N>_<workload>.json
set -o pipefail
export TMPDIR=/tmp
T=$1; N=$2; W=${3:-cfg4}
O=gpurun_out/$T; mkdir -p $O
timeout -k 10 600 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node $N --master-addr 127.0.0.1 \
    --master-port $((29500 + N)) bench.py --gpus $N --dist-backend gloo --workload $W --steps 3 --warmup 1 \
    > $O/n${N}_$W.raw 2> $O/n${N}_$W.err || exit 1
grep '^{' $O/n${N}_$W.raw > $O/n${N}_$W.json
python3 -c "import json; d=json.load(open('$O/n${N}_$W.json')); print('N=$N $W', d['value'], d['unit'], 'selfcheck', d.get('topk_selfcheck'), d['config']['parallelism'])"
