# final tree: full GPU suite + smoke
set -o pipefail
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out/r8p
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 600 --timeout-method thread > gpurun_out/r8p/gputest.log 2>&1 || exit 1
timeout -k 10 240 python3 -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r8p/smoke.log 2>&1 || exit 2
