#!/bin/bash
# A/B of the phase-B unit size on configs[2] (1e9 rows). TAG names outputs.
set -o pipefail
cd "$(dirname "$0")/.." || exit 1
export TMPDIR=/tmp
O=gpurun_out
T=${TAG:-r2}
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_freq.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/gpu_freq_only_$T.log 2>&1 &&
for U in 2 8 32; do
  DQ_FREQ_UNIT_TILES=$U timeout -k 10 300 python -u tools/bench_workloads.py c3 --steps 3 > $O/wl_c3_u${U}_$T.json 2>&1 || exit 1
done
