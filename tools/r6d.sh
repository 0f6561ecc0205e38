# round-5: ticket-mode A/B, the GPU suite (DPP scans; the new full-size 1024-query batch test), PC sampling
set -o pipefail
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out/r6d
bash tools/gpu_round.sh r6d quick quickv:relaxed quickv:acqrel || exit 1
cp gpurun_out/r6d/quick.json gpurun_out/r6d/quick_a.json
bash tools/gpu_round.sh r6d quick tests || exit 2
timeout -k 10 240 rocprofv3 --pc-sampling-beta-enabled --pc-sampling-method stochastic --pc-sampling-unit cycles --pc-sampling-interval 1048576 -d gpurun_out/r6d/pcs -o run -- python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-pmc --no-cfg3 > gpurun_out/r6d/pcs.json 2> gpurun_out/r6d/pcs.err || exit 3
