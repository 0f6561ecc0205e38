# final K1' counter passes on cfg 3 (separate rocprofv3 --pmc runs, one counter group each)
set -o pipefail
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp
bash tools/pmc_passes.sh r3al_k1p fas_pairs --workload cfg3 > gpurun_out/r3al_pmc.log 2>&1 || exit 1
