#!/bin/bash
# GPU test session: TESTS (default: the whole -m gpu suite), output gpurun_out/gpu_tests_$TAG.log
set -o pipefail
cd "$(dirname "$0")/.." || exit 1
export TMPDIR=/tmp
O=gpurun_out
T=${TAG:-r2}
mkdir -p $O
timeout -k 10 ${LIMIT:-500} python -u -m pytest ${TESTS:-tests} -m gpu -x -v --timeout 120 --timeout-method thread > $O/gpu_tests_$T.log 2>&1
