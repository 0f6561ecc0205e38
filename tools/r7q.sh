# final tree: GPU suite (incl. the primitive probe), the default bench line, rocprof stats
set -o pipefail
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out/r7q
bash tools/gpu_round.sh r7q tests bench prof || exit 1
