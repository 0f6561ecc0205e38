# final tree after the ping-pong streams: the default bench line, cfg 3 and cfg 5 lines, rocprof stats
set -o pipefail
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out/r7zz
bash tools/gpu_round.sh r7zz bench prof cfg3 cfg5 || exit 1
