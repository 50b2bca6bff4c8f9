#!/bin/bash
# PMC passes over configs[4] (one step, no warmup; one counter set per rocprofv3 run): HBM bytes per
# kernel (FETCH_SIZE, WRITE_SIZE), then wave-state and instruction-mix SQ counters.
# Summarise with: python tools/summarize_c3_pmc.py TAG c5
set -o pipefail
cd "$(dirname "$0")/.." || exit 1
export TMPDIR=/tmp
O=gpurun_out
T=${TAG:-r4}
W="tools/bench_workloads.py c5 --steps 1 --warmup 0"
mkdir -p $O
timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/pmcf_c5_$T -o run -- python3 $W > $O/pmcf_c5_$T.log 2>&1 &&
timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/pmcw_c5_$T -o run -- python3 $W > $O/pmcw_c5_$T.log 2>&1 &&
timeout -s KILL 240 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_INSTS_VALU --output-format csv -d $O/pmc_c5_$T -o sq -- python3 $W > $O/pmc_c5_$T.log 2>&1 &&
timeout -s KILL 240 rocprofv3 --pmc SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SALU SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_SMEM SQ_IFETCH SQ_WAIT_INST_ANY --output-format csv -d $O/pmc2_c5_$T -o sq -- python3 $W > $O/pmc2_c5_$T.log 2>&1
