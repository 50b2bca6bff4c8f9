#!/bin/bash
# S10 evidence session: the bench line, its rocprofv3 kernel stats, then the FETCH_SIZE and
# WRITE_SIZE PMC passes (one counter group per run, as the guide prescribes) of the same command.
# Summarise afterwards with: python tools/summarize_profile.py $TAG
set -o pipefail
cd "$(dirname "$0")/.." || exit 1
export TMPDIR=/tmp
O=gpurun_out
T=${TAG:-r3}
mkdir -p $O
timeout -k 10 300 python -u bench.py --steps 20 --warmup 3 > $O/bench_$T.json 2> $O/bench_$T.err &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_$T -o run -- python3 bench.py --steps 10 --warmup 2 --no-h2d --no-cpu-baseline --workloads '' > $O/prof_$T.log 2>&1 &&
timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/pmc_fetch_$T -o run -- python3 bench.py --steps 3 --warmup 1 --no-h2d --no-cpu-baseline --workloads '' > $O/pmc_fetch_$T.log 2>&1 &&
timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/pmc_write_$T -o run -- python3 bench.py --steps 3 --warmup 1 --no-h2d --no-cpu-baseline --workloads '' > $O/pmc_write_$T.log 2>&1
