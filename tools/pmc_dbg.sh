#!/bin/bash
# usage: tools/pmc_dbg.sh <tag> <kernel-regex> <dbg values...>
# one rocprofv3 --pmc pass of instruction counters per PF_K5_DBG value (phases switched off;
# profiling only, scores are wrong then): attributes the scan kernel's instructions to phases
set -o pipefail
export TMPDIR=/tmp
T=$1; K=$2; shift; shift
mkdir -p gpurun_out/dbg_$T
for d in "$@"; do
  PF_K5_DBG=$d timeout -k 10 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY GRBM_GUI_ACTIVE \
    --kernel-include-regex $K -T --output-format csv -d gpurun_out/dbg_$T/d$d -o run -- \
    python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-pmc > gpurun_out/dbg_$T/d$d.log 2>&1 || exit 1
done
