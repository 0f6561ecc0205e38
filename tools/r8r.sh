# batch default 32: full GPU suite + cfg 4 line
set -o pipefail
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out/r8r
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 600 --timeout-method thread > gpurun_out/r8r/gputest.log 2>&1 || exit 1
timeout -k 10 300 python3 bench.py --workload cfg4 --steps 4 --warmup 1 --no-pmc --no-cpu-baseline > gpurun_out/r8r/cfg4.json 2> gpurun_out/r8r/cfg4.err || exit 2
