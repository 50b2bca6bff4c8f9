#!/bin/bash
# Round 6, configs[4] string phase A: the arena copy measured.  Kernel stats of one step under the
# default build, a build whose phase A writes no arena key bytes (abl/libdq_anocopy.so, timing
# only); then FETCH_SIZE / WRITE_SIZE passes of both.  (A third build, hashed phase C's compares
# behind one more dependent load -- a column reference's offsets hop -- stopped answering on the
# box, r6p, and was dropped.)  TIMING_LIBS=none skips the timing leg.  TAG names the outputs.
set -o pipefail
cd "$(dirname "$0")/.." || exit 1
export TMPDIR=/tmp
O=gpurun_out
T=${TAG:-r6}
W="tools/bench_workloads.py c5 --steps 1 --warmup 1"
mkdir -p $O
i=0
for L in ${TIMING_LIBS-"" abl/libdq_anocopy.so}; do
  [ "$L" = none ] && break
  DQ_LIB_PATH=$L timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/c5ab_${T}_$i -o run -- python3 $W > $O/c5ab_${T}_$i.log 2>&1 || exit 1
  i=$((i+1))
done
i=0
for L in "" abl/libdq_anocopy.so; do
  DQ_LIB_PATH=$L timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/c5f_${T}_$i -o run -- python3 tools/bench_workloads.py c5 --steps 1 --warmup 0 > $O/c5f_${T}_$i.log 2>&1 || exit 1
  DQ_LIB_PATH=$L timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/c5w_${T}_$i -o run -- python3 tools/bench_workloads.py c5 --steps 1 --warmup 0 > $O/c5w_${T}_$i.log 2>&1 || exit 1
  i=$((i+1))
done
