set -o pipefail
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out/r7x
bash tools/gpu_round.sh r7x quick quicke:k5_wgs=800 quicke:k5_wgs=896 quicke:k5_wgs=960 quicke:k5_dyn=1 quicke:k5_tail=256 quick || exit 1
