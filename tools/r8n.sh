set -o pipefail
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && O=gpurun_out/r8n && mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -v -m gpu --timeout 120 --timeout-method thread -k "sharded or scan_lanes" > $O/tests.log 2>&1 || exit 1
