#!/bin/bash
# Round 6 A/B: group-by tests, then configs[2] timed under each env setting in $AB (";"-separated,
# "-" = defaults), then one DQ_FREQ_DEBUG=2 pass.  TAG names the outputs.
set -o pipefail
cd "$(dirname "$0")/.." || exit 1
export TMPDIR=/tmp
O=gpurun_out
T=${TAG:-r6}
mkdir -p $O
timeout -k 10 500 python -u -m pytest ${TESTS:-tests/test_gpu_freq.py tests/test_gpu_fullsize_dups.py} -x -v --timeout 300 --timeout-method thread > $O/gpu_tests_$T.log 2>&1 || exit 1
IFS=';' read -ra SETS <<< "${AB:--}"
i=0
for e in "${SETS[@]}"; do
  [ "$e" = "-" ] && e=""
  env $e timeout -k 10 200 python -u tools/bench_workloads.py ${WL:-c3} --steps ${STEPS:-8} > $O/wl_${WL:-c3}_${T}_$i.json 2>&1 || exit 1
  if [ -n "$PROF" ]; then
    env $e timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_${T}_$i -o run -- python3 tools/bench_workloads.py ${WL:-c3} --steps ${PSTEPS:-3} > $O/prof_${T}_$i.log 2>&1 || exit 1
  fi
  echo "$i: $e" >> $O/ab_$T.txt
  i=$((i+1))
done
if [ -n "$DBG" ]; then
  DQ_FREQ_DEBUG=2 timeout -k 10 200 python -u tools/bench_workloads.py ${WL:-c3} --steps 1 --warmup 0 > $O/dbg_${WL:-c3}_$T.log 2>&1 || exit 1
fi
