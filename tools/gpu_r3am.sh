# the driver's round-end sequence on the final tree: smoke(), then the default bench line
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/r3am && export TMPDIR=/tmp
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r3am/smoke.log 2>&1 || exit 1
timeout -k 10 600 python3 bench.py > gpurun_out/r3am/bench.json 2> gpurun_out/r3am/bench.err || exit 2
