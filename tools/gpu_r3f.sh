set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/r3f && export TMPDIR=/tmp
timeout -k 10 300 python3 bench.py --workload cfg3 --steps 60 --warmup 5 --no-cpu-baseline --no-pmc > gpurun_out/r3f/cfg3.json 2> gpurun_out/r3f/cfg3.err || exit 2
make -C recommendation-system-pokec_amd clean > /dev/null && make -C recommendation-system-pokec_amd -j16 K5T=1 > gpurun_out/r3f/build_k5t.log 2>&1 || exit 3
timeout -k 10 300 python3 bench.py --workload cfg3 --steps 30 --warmup 3 --no-cpu-baseline --no-pmc > gpurun_out/r3f/cfg3_k5t.json 2> gpurun_out/r3f/cfg3_k5t.err || exit 4
