# round-3 final profiles: rocprof kernel stats of the default run, K5 / K1' counter passes, an
# N=2 rehearsal on one GPU over gloo (the n1_same_workload field), the full GPU suite
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/r3r && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r3r/prof_default -o run -- python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-pmc > gpurun_out/r3r/default_prof.json 2> gpurun_out/r3r/default_prof.err || exit 1
bash tools/pmc_passes.sh r3r_k5 fas_post > gpurun_out/r3r/pmc_k5.log 2>&1 || exit 2
timeout -k 10 600 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 2 --dist-backend gloo --steps 5 --warmup 2 --no-pmc > gpurun_out/r3r/rehearsal_n2_gloo.json 2> gpurun_out/r3r/rehearsal_n2_gloo.err || exit 3
timeout -k 10 1100 python -u -m pytest tests -m gpu -x -v -s --timeout 600 --timeout-method thread > gpurun_out/r3r/gputest_full.log 2>&1 || exit 4
