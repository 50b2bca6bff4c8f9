#!/bin/bash
# Round-5 sessions; TAG names outputs, PART selects the steps.  Every GPU step runs under its own
# time limit and the steps are chained with &&: a failure, fault or time-out ends the session.
#  PART=full:  the stated-size checks (tests/test_gpu_fullsize.py), the whole -m gpu suite, then
#              the S10 evidence session (tools/gpu_s10_prof.sh: bench line, kernel stats,
#              FETCH_SIZE / WRITE_SIZE passes).
#  PART=tests: the -m gpu suite only (TESTS narrows it).
#  PART=all:   the whole -m gpu suite, then the configs[4] line with its CPU baseline and the
#              configs[2] / [3] lines.
#  PART=wl:    configs[2] / [3] / [4] lines (tools/bench_workloads.py).
#  PART=c3:    configs[2] line, its rocprof kernel stats and PMC passes (tools/gpu_pmc_c3.sh).
#  PART=s10ab: parity tests, then scan ablation + bench of this build against the build at $VAR.
#  PART=pmc:   the configs[2] and configs[4] PMC passes (tools/gpu_pmc_c3.sh, gpu_pmc_c5.sh).
#  PART=dense: the group-by tests with the dense integer path, configs[4] with and without it,
#              configs[2], and configs[4]'s kernel stats.
#  PART=hll:   the HLL-from-table tests, configs[4] with and without it.
#  PART=c5:    configs[4] line and its rocprof kernel stats.
set -o pipefail
cd "$(dirname "$0")/.." || exit 1
export TMPDIR=/tmp
O=gpurun_out
T=${TAG:-r5}
mkdir -p $O
PYT="python -u -m pytest -x -v --timeout 300 --timeout-method thread"
case "${PART:-full}" in
full)
  timeout -k 10 600 $PYT tests/test_gpu_fullsize.py > $O/gpu_fullsize_$T.log 2>&1 &&
  timeout -k 10 700 $PYT tests -m gpu --ignore=tests/test_gpu_fullsize.py > $O/gpu_tests_$T.log 2>&1 &&
  TAG=$T bash tools/gpu_s10_prof.sh
  ;;
tests)
  timeout -k 10 ${LIMIT:-800} $PYT ${TESTS:-tests} -m gpu > $O/gpu_tests_$T.log 2>&1
  ;;
all)
  timeout -k 10 800 $PYT tests -m gpu > $O/gpu_tests_$T.log 2>&1 &&
  timeout -k 10 200 python -u bench.py --no-cpu-baseline > $O/bench_$T.json 2>&1 &&
  DQ_TAIL_SPLIT=0 timeout -k 10 200 python -u bench.py --no-cpu-baseline --no-h2d > $O/bench_notail_$T.json 2>&1 &&
  timeout -k 10 200 python -u bench.py --no-cpu-baseline --no-h2d > $O/bench2_$T.json 2>&1 &&
  timeout -k 10 500 python -u tools/bench_workloads.py c5 --steps 5 --cpu-baseline --cpu-rows 8388608 > $O/wl_c5_$T.json 2>&1 &&
  timeout -k 10 300 python -u tools/bench_workloads.py c3 --steps 5 > $O/wl_c3_$T.json 2>&1 &&
  timeout -k 10 300 python -u tools/bench_workloads.py c4 --steps 10 --warmup 3 > $O/wl_c4_$T.json 2>&1 &&
  DQ_FREQ_PARTITION_TARGET=3800 timeout -k 10 300 python -u tools/bench_workloads.py c3 --steps 5 > $O/wl_c3_t3800_$T.json 2>&1 &&
  DQ_TAIL_SPLIT=0 timeout -k 10 300 python -u tools/bench_workloads.py c4 --steps 10 --warmup 3 > $O/wl_c4_notail_$T.json 2>&1
  ;;
ab)
  timeout -k 10 800 $PYT tests -m gpu > $O/gpu_tests_$T.log 2>&1 || exit 1
  for k in 1 2; do
    DQ_TAIL_SPLIT=0 timeout -k 10 200 python -u bench.py --no-cpu-baseline --no-h2d > $O/bench_notail${k}_$T.json 2>&1 &&
    timeout -k 10 200 python -u bench.py --no-cpu-baseline --no-h2d > $O/bench_tail${k}_$T.json 2>&1 &&
    DQ_EAGER_RESET=1 timeout -k 10 200 python -u bench.py --no-cpu-baseline --no-h2d > $O/bench_eager${k}_$T.json 2>&1 || exit 1
  done
  DQ_HLL_FROM_TABLE=0 timeout -k 10 400 python -u tools/bench_workloads.py c5 --steps 5 > $O/wl_c5_nohll_$T.json 2>&1 &&
  timeout -k 10 400 python -u tools/bench_workloads.py c5 --steps 5 > $O/wl_c5_$T.json 2>&1 &&
  timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_c5_$T -o run -- python3 tools/bench_workloads.py c5 --steps 2 > $O/prof_c5_$T.log 2>&1
  ;;
wl)
  timeout -k 10 300 python -u tools/bench_workloads.py c3 --steps 5 > $O/wl_c3_$T.json 2>&1 &&
  timeout -k 10 300 python -u tools/bench_workloads.py c4 --steps 10 --warmup 3 > $O/wl_c4_$T.json 2>&1 &&
  timeout -k 10 400 python -u tools/bench_workloads.py c5 --steps 5 > $O/wl_c5_$T.json 2>&1
  ;;
c3)
  timeout -k 10 300 python -u tools/bench_workloads.py c3 --steps 5 > $O/wl_c3_$T.json 2>&1 &&
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_c3_$T -o run -- python3 tools/bench_workloads.py c3 --steps 2 > $O/prof_c3_$T.log 2>&1 &&
  TAG=$T bash tools/gpu_pmc_c3.sh
  ;;
s10ab)
  # A/B of a scan-body variant built at $VAR (DQ_LIB_PATH: diagnostic builds only)
  timeout -k 10 300 $PYT tests/test_gpu_parity.py tests/test_gpu_configs4.py tests/test_gpu_freq.py > $O/gpu_tests_$T.log 2>&1 &&
  timeout -k 10 300 python -u tools/bench_workloads.py c3 --steps 5 > $O/wl_c3_new_$T.json 2>&1 &&
  DQ_LIB_PATH=$VAR timeout -k 10 300 python -u tools/bench_workloads.py c3 --steps 5 > $O/wl_c3_var_$T.json 2>&1 &&
  for k in 1 2; do
    timeout -k 10 200 python -u tools/scan_ablation.py > $O/abl_new${k}_$T.log 2>&1 &&
    DQ_LIB_PATH=$VAR timeout -k 10 200 python -u tools/scan_ablation.py > $O/abl_var${k}_$T.log 2>&1 &&
    timeout -k 10 200 python -u bench.py --no-cpu-baseline --no-h2d > $O/bench_new${k}_$T.json 2>&1 &&
    DQ_LIB_PATH=$VAR timeout -k 10 200 python -u bench.py --no-cpu-baseline --no-h2d > $O/bench_var${k}_$T.json 2>&1 || exit 1
  done
  ;;
pmc)
  TAG=$T bash tools/gpu_pmc_c3.sh && TAG=$T bash tools/gpu_pmc_c5.sh
  ;;
dense)
  timeout -k 10 400 $PYT ${TESTS:-tests/test_gpu_freq_dense.py tests/test_gpu_freq.py tests/test_gpu_configs4.py tests/test_gpu_hll_tables.py tests/test_gpu_determinism.py} > $O/gpu_tests_$T.log 2>&1 &&
  timeout -k 10 400 python -u tools/bench_workloads.py c5 --steps 5 > $O/wl_c5_$T.json 2>&1 &&
  env ${AB:-DQ_FREQ_DENSE=0} timeout -k 10 400 python -u tools/bench_workloads.py c5 --steps 5 > $O/wl_c5_nodense_$T.json 2>&1 &&
  timeout -k 10 300 python -u tools/bench_workloads.py c3 --steps 5 > $O/wl_c3_$T.json 2>&1 &&
  env ${AB:-DQ_FREQ_DENSE=0} timeout -k 10 300 python -u tools/bench_workloads.py c3 --steps 5 > $O/wl_c3_ab_$T.json 2>&1 &&
  timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_c5_$T -o run -- python3 tools/bench_workloads.py c5 --steps 2 > $O/prof_c5_$T.log 2>&1
  ;;
hll)
  timeout -k 10 300 $PYT tests/test_gpu_hll_tables.py tests/test_gpu_determinism.py > $O/gpu_tests_$T.log 2>&1 &&
  DQ_HLL_FROM_TABLE=0 timeout -k 10 400 python -u tools/bench_workloads.py c5 --steps 5 > $O/wl_c5_nohll_$T.json 2>&1 &&
  timeout -k 10 400 python -u tools/bench_workloads.py c5 --steps 5 > $O/wl_c5_$T.json 2>&1 &&
  DQ_HLL_TABLE_RECORDS_PER_ROW=1 timeout -k 10 400 python -u tools/bench_workloads.py c5 --steps 5 > $O/wl_c5_q_$T.json 2>&1 &&
  timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_c5_$T -o run -- python3 tools/bench_workloads.py c5 --steps 2 > $O/prof_c5_$T.log 2>&1
  ;;
c5)
  timeout -k 10 400 python -u tools/bench_workloads.py c5 --steps 5 > $O/wl_c5_$T.json 2>&1 &&
  timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_c5_$T -o run -- python3 tools/bench_workloads.py c5 --steps 2 > $O/prof_c5_$T.log 2>&1
  ;;
esac
