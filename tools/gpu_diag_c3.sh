#!/bin/bash
# configs[2] diagnostics: DQ_FREQ_DEBUG=2 per-phase stamps (workgroup 0) at 1e9 rows, then SQ
# instruction / wait counters of the group-by kernels at 1e8 rows.  TAG names the outputs.
set -o pipefail
cd "$(dirname "$0")/.." || exit 1
export TMPDIR=/tmp
O=gpurun_out
T=${TAG:-diag}
W="tools/bench_workloads.py c3 --rows 100000000 --steps 1 --warmup 0"
mkdir -p $O
DQ_FREQ_DEBUG=2 timeout -k 10 300 python -u tools/bench_workloads.py c3 --steps 1 --warmup 0 > $O/dbg_c3_$T.log 2>&1 &&
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_INSTS_VALU --output-format csv -d $O/pmc_c3_$T -o sq -- python3 $W > $O/pmc_c3_$T.log 2>&1 &&
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SALU SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_SMEM SQ_IFETCH SQ_BUSY_CYCLES --output-format csv -d $O/pmc2_c3_$T -o sq -- python3 $W > $O/pmc2_c3_$T.log 2>&1
