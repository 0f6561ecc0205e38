#!/bin/bash
# usage: tools/pmc_passes.sh <tag> [kernel-regex] [extra bench args...]
# separate rocprofv3 --pmc passes (one counter group per run) over a short bench;
# tools/pmc_summary.py --sq summarises them per launch
set -o pipefail
export TMPDIR=/tmp
T=$1
K=${2:-fas_post}
shift; shift
B="python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-pmc $*"
run() { timeout -k 10 120 rocprofv3 --pmc $2 --kernel-include-regex $K -T --output-format csv -d gpurun_out/pmc_$T/$1 -o run -- $B > gpurun_out/pmc_$T/$1.log 2>&1; echo "$1 rc=$?"; }
mkdir -p gpurun_out/pmc_$T
run p1 "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE" &&
run p2 "SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INST_LEVEL_VMEM" &&
run p3 "FETCH_SIZE" &&
run p4 "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INST_LEVEL_LDS SQ_WAIT_INST_LDS SQ_INSTS_SMEM SQ_INSTS_VALU_FP64" &&
run p5 "TA_BUSY_avr TCP_TOTAL_CACHE_ACCESSES_sum TCC_HIT_sum TCC_MISS_sum"
