# round-5: K5 phase-skip timings (vlib/no*) and the VALU instruction mix
set -o pipefail
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out/r6l
bash tools/gpu_round.sh r6l quick quickv:noterms quickv:noitems quickv:nofas quickv:noowner quickv:noplace quickv:nomerge quickv:nosets quickv:notext quick || exit 1
bash tools/gpu_round.sh r6l pmc:mix:SQ_INSTS_VALU_INT32,SQ_INSTS_VALU_INT64,SQ_INSTS_VALU_CVT,SQ_INSTS_VALU_ADD_F64,SQ_INSTS_VALU_MUL_F64,SQ_INSTS_VALU_FMA_F64,SQ_INSTS_VALU_TRANS_F64,SQ_INSTS_VALU_TRANS_F32 || exit 2
