set -o pipefail
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out/r7k
bash tools/gpu_round.sh r7k quick4 quick4e:k5_batch_blocks=8 quick4e:k5_batch_blocks=32 quick4e:k5_batch_blocks=12 quick4e:k5_batch_blocks=24 quick4 || exit 1
