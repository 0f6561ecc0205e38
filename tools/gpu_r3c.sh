set -o pipefail
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp
bash tools/pmc_passes.sh r3c_k1p fas_pairs --workload cfg3 --contexts 1 || exit 1
bash tools/pmc_passes.sh r3c_k5 fas_post --no-cfg3 || exit 2
python3 tools/pmc_sq.py gpurun_out/pmc_r3c_k1p fas_pairs_kernel > gpurun_out/pmc_r3c_k1p/summary.json
python3 tools/pmc_sq.py gpurun_out/pmc_r3c_k5 fas_post_kernel > gpurun_out/pmc_r3c_k5/summary.json
