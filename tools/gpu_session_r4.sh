#!/bin/bash
# Round-4 sessions; TAG names outputs, PART selects the half.
#  PART=1: the whole -m gpu suite, S10 bench (A/B of the mixed-kernel mask), configs[2]/[3] lines
#          with their CPU baselines, and configs[2] with the generic phase-A kernel (A/B).
#  PART=2: the multi-GPU harness rehearsed as 2 ranks on one GPU, rocprof kernel stats of
#          configs[2] and configs[4], and the configs[4] line with its CPU baseline.
set -o pipefail
cd "$(dirname "$0")/.." || exit 1
export TMPDIR=/tmp
O=gpurun_out
T=${TAG:-s}
mkdir -p $O
if [ "${PART:-1}" = 1 ]; then
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gpu_tests_$T.log 2>&1 &&
timeout -k 10 120 python -u bench.py > $O/bench_$T.json 2>&1 &&
DQ_MIXED_ALL=1 timeout -k 10 120 python -u bench.py > $O/bench_all_$T.json 2>&1 &&
timeout -k 10 400 python -u tools/bench_workloads.py c3 --steps 3 --cpu-baseline > $O/wl_c3_$T.json 2>&1 &&
DQ_FREQ_GENERIC_A=1 timeout -k 10 300 python -u tools/bench_workloads.py c3 --steps 3 > $O/wl_c3_genA_$T.json 2>&1 &&
timeout -k 10 300 python -u tools/bench_workloads.py c4 --steps 5 --cpu-baseline > $O/wl_c4_$T.json 2>&1 &&
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_c5_$T -o run -- python3 tools/bench_workloads.py c5 --steps 2 > $O/prof_c5_$T.log 2>&1 &&
DQ_FREQ_DEBUG=2 timeout -k 10 300 python -u tools/bench_workloads.py c5 --steps 1 --warmup 0 > $O/dbg_c5_$T.log 2>&1
elif [ "${PART}" = 4 ]; then
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gpu_tests_$T.log 2>&1 &&
timeout -k 10 400 python -u tools/bench_workloads.py c5 --steps 3 > $O/wl_c5_$T.json 2>&1 &&
DQ_RX_ROWS=2 timeout -k 10 400 python -u tools/bench_workloads.py c5 --steps 3 > $O/wl_c5rx2_$T.json 2>&1 &&
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_c5_$T -o run -- python3 tools/bench_workloads.py c5 --steps 2 > $O/prof_c5_$T.log 2>&1 &&
DQ_FREQ_DEBUG=2 timeout -k 10 300 python -u tools/bench_workloads.py c5 --steps 1 --warmup 0 > $O/dbg_c5_$T.log 2>&1 &&
timeout -k 10 300 python -u tools/bench_workloads.py c3 --steps 3 > $O/wl_c3_$T.json 2>&1 &&
timeout -k 10 300 python -u tools/bench_workloads.py c4 --steps 10 --warmup 3 > $O/wl_c4_$T.json 2>&1
elif [ "${PART}" = 5 ]; then
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gpu_tests_$T.log 2>&1 &&
timeout -k 10 400 python -u tools/bench_workloads.py c5 --steps 3 > $O/wl_c5_$T.json 2>&1 &&
timeout -k 10 400 python -u tools/bench_workloads.py c5 --steps 1 --pyprof > $O/pyprof_c5_$T.log 2>&1 &&
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_c5_$T -o run -- python3 tools/bench_workloads.py c5 --steps 2 > $O/prof_c5_$T.log 2>&1 &&
DQ_FREQ_DEBUG=2 timeout -k 10 300 python -u tools/bench_workloads.py c3 --steps 1 --warmup 1 > $O/dbg_c3_$T.log 2>&1 &&
timeout -k 10 300 python -u tools/bench_workloads.py c3 --steps 3 > $O/wl_c3_$T.json 2>&1
elif [ "${PART}" = 6 ]; then
timeout -k 10 300 python -u -m pytest tests/test_gpu_pattern_quantile.py tests/test_gpu_configs4.py -x -q --timeout 200 --timeout-method thread > $O/gpu_tests_q_$T.log 2>&1 &&
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_c5_$T -o run -- python3 tools/bench_workloads.py c5 --steps 2 > $O/prof_c5_$T.log 2>&1 &&
timeout -k 10 400 python -u tools/bench_workloads.py c5 --steps 3 > $O/wl_c5_$T.json 2>&1 &&
DQ_RUN_WORKERS=2 DQ_RUN_TRACE=1 timeout -k 10 400 python -u tools/bench_workloads.py c5 --steps 3 > $O/wl_c5w2_$T.json 2>&1 &&
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gpu_tests_$T.log 2>&1
elif [ "${PART}" = 7 ]; then
timeout -k 10 300 python -u -m pytest tests/test_gpu_pattern_quantile.py tests/test_gpu_configs4.py -x -q --timeout 200 --timeout-method thread > $O/gpu_tests_q_$T.log 2>&1 &&
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_c5_$T -o run -- python3 tools/bench_workloads.py c5 --steps 2 > $O/prof_c5_$T.log 2>&1 &&
timeout -k 10 400 python -u tools/bench_workloads.py c5 --steps 3 > $O/wl_c5_$T.json 2>&1
elif [ "${PART}" = 8 ]; then
timeout -k 10 300 python -u -m pytest tests/test_gpu_datatype_mi.py tests/test_gpu_configs4.py -x -q --timeout 200 --timeout-method thread > $O/gpu_tests_q_$T.log 2>&1 &&
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_c5_$T -o run -- python3 tools/bench_workloads.py c5 --steps 2 > $O/prof_c5_$T.log 2>&1 &&
timeout -k 10 400 python -u tools/bench_workloads.py c5 --steps 3 > $O/wl_c5_$T.json 2>&1 &&
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gpu_tests_$T.log 2>&1
elif [ "${PART}" = 9 ]; then
timeout -k 10 400 python -u -m pytest tests/test_gpu_datatype_mi.py tests/test_gpu_configs4.py tests/test_gpu_freq.py -x -v --timeout 200 --timeout-method thread > $O/gpu_tests_q_$T.log 2>&1 &&
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_c5_$T -o run -- python3 tools/bench_workloads.py c5 --steps 2 > $O/prof_c5_$T.log 2>&1 &&
timeout -k 10 400 python -u tools/bench_workloads.py c5 --steps 3 > $O/wl_c5_$T.json 2>&1 &&
DQ_FREQ_DEBUG=2 timeout -k 10 300 python -u tools/bench_workloads.py c3 --steps 1 --warmup 1 > $O/dbg_c3_$T.log 2>&1 &&
timeout -k 10 300 python -u tools/bench_workloads.py c3 --steps 5 > $O/wl_c3_$T.json 2>&1 &&
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gpu_tests_$T.log 2>&1
elif [ "${PART}" = 10 ]; then
timeout -k 10 400 python -u -m pytest tests/test_gpu_datatype_mi.py tests/test_gpu_freq.py -x -q --timeout 200 --timeout-method thread > $O/gpu_tests_q_$T.log 2>&1 &&
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_c5_$T -o run -- python3 tools/bench_workloads.py c5 --steps 2 > $O/prof_c5_$T.log 2>&1 &&
timeout -k 10 400 python -u tools/bench_workloads.py c5 --steps 3 > $O/wl_c5_$T.json 2>&1 &&
DQ_FREQ_DEBUG=2 timeout -k 10 300 python -u tools/bench_workloads.py c5 --steps 1 --warmup 0 > $O/dbg_c5_$T.log 2>&1
elif [ "${PART}" = 11 ]; then
timeout -k 10 400 python -u -m pytest tests/test_gpu_freq.py tests/test_gpu_configs4.py -x -q --timeout 200 --timeout-method thread > $O/gpu_tests_q_$T.log 2>&1 &&
TAG=$T bash tools/gpu_s10_prof.sh &&
TAG=$T bash tools/gpu_pmc_c3.sh &&
timeout -k 10 300 python -u tools/bench_workloads.py c4 --steps 10 --warmup 3 > $O/wl_c4_$T.json 2>&1 &&
timeout -k 10 300 python -u tools/bench_workloads.py c3 --steps 5 > $O/wl_c3_$T.json 2>&1 &&
timeout -k 10 400 python -u tools/bench_workloads.py c5 --steps 3 > $O/wl_c5_$T.json 2>&1
elif [ "${PART}" = 12 ]; then
timeout -k 10 400 python -u -m pytest tests/test_gpu_freq.py -x -q --timeout 200 --timeout-method thread -k "topk or Histogram or histogram" > $O/gpu_tests_k_$T.log 2>&1 &&
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_c5_$T -o run -- python3 tools/bench_workloads.py c5 --steps 2 > $O/prof_c5_$T.log 2>&1 &&
timeout -k 10 400 python -u tools/bench_workloads.py c5 --steps 3 > $O/wl_c5_$T.json 2>&1 &&
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gpu_tests_$T.log 2>&1
elif [ "${PART}" = 13 ]; then
timeout -k 10 400 python -u tools/bench_workloads.py c5 --steps 3 > $O/wl_c5_$T.json 2>&1 &&
DQ_RUN_WORKERS=2 timeout -k 10 400 python -u tools/bench_workloads.py c5 --steps 3 > $O/wl_c5w2_$T.json 2>&1 &&
DQ_RUN_WORKERS=3 timeout -k 10 400 python -u tools/bench_workloads.py c5 --steps 3 > $O/wl_c5w3_$T.json 2>&1 &&
timeout -k 10 400 python -u tools/bench_workloads.py c5 --steps 1 --pyprof > $O/pyprof_c5_$T.log 2>&1 &&
DQ_RUN_TRACE=1 timeout -k 10 400 python -u tools/bench_workloads.py c5 --steps 1 > $O/trace_c5_$T.log 2>&1
elif [ "${PART}" = 15 ]; then
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke_$T.log 2>&1 &&
timeout -k 10 200 python -u bench.py > $O/bench_$T.json 2>&1 &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_s10_$T -o run -- python3 bench.py --steps 20 > $O/prof_s10_$T.log 2>&1 &&
timeout -k 10 300 python -u tools/bench_workloads.py c3 --steps 3 > $O/wl_c3_$T.json 2>&1 &&
timeout -k 10 300 python -u tools/bench_workloads.py c4 --steps 10 --warmup 3 > $O/wl_c4_$T.json 2>&1
elif [ "${PART}" = 14 ]; then
timeout -k 10 400 python -u -m pytest tests/test_gpu_datatype_mi.py tests/test_gpu_configs4.py -x -q --timeout 200 --timeout-method thread > $O/gpu_tests_q_$T.log 2>&1 &&
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_c5_$T -o run -- python3 tools/bench_workloads.py c5 --steps 2 > $O/prof_c5_$T.log 2>&1 &&
timeout -k 10 400 python -u tools/bench_workloads.py c5 --steps 3 > $O/wl_c5_$T.json 2>&1 &&
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gpu_tests_$T.log 2>&1
elif [ "${PART}" = 3 ]; then
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gpu_tests_$T.log 2>&1 &&
timeout -k 10 400 python -u tools/bench_workloads.py c5 --steps 3 > $O/wl_c5_$T.json 2>&1 &&
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_c5_$T -o run -- python3 tools/bench_workloads.py c5 --steps 2 > $O/prof_c5_$T.log 2>&1 &&
DQ_FREQ_DEBUG=2 timeout -k 10 300 python -u tools/bench_workloads.py c5 --steps 1 --warmup 0 > $O/dbg_c5_$T.log 2>&1 &&
timeout -k 10 300 python -u tools/bench_workloads.py c3 --steps 3 > $O/wl_c3_$T.json 2>&1 &&
timeout -k 10 300 python -u tools/bench_workloads.py c4 --steps 10 --warmup 3 > $O/wl_c4_$T.json 2>&1
else
timeout -k 10 300 python -u tools/bench_workloads.py c3 --rows 100000000 --steps 2 --warmup 1 --gpus 2 --share-gpu > $O/dist_c3_$T.json 2>&1 &&
timeout -k 10 300 python -u tools/bench_workloads.py c4 --rows 100000000 --steps 2 --warmup 1 --gpus 2 --share-gpu > $O/dist_c4_$T.json 2>&1 &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_c3_$T -o run -- python3 tools/bench_workloads.py c3 --steps 2 > $O/prof_c3_$T.log 2>&1 &&
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_c5_$T -o run -- python3 tools/bench_workloads.py c5 --steps 2 > $O/prof_c5_$T.log 2>&1 &&
timeout -k 10 400 python -u tools/bench_workloads.py c5 --steps 3 --cpu-baseline --cpu-rows 8388608 > $O/wl_c5_$T.json 2>&1
fi
