set -o pipefail
cd /root/repo
O=gpurun_out; mkdir -p $O
PYT="python -u -m pytest -x -v --timeout 300 --timeout-method thread"
timeout -k 10 400 $PYT tests/test_gpu_freq.py tests/test_gpu_configs4.py > $O/gpu_tests_pf.log 2>&1 &&
for k in 1 2; do
  timeout -k 10 300 python -u tools/bench_workloads.py c3 --steps 5 > $O/wl_c3_pf$k.json 2>&1 &&
  DQ_LIB_PATH=var_base/libdeequ_amd.so timeout -k 10 300 python -u tools/bench_workloads.py c3 --steps 5 > $O/wl_c3_base$k.json 2>&1 || exit 1
done
