#!/usr/bin/env bash
set -o pipefail
# nbx_perf C-driver tests, then -m 1 vs -m 16 aggregation (profiles/r1/nbx_perf_agg_*.txt)
cd "${GRAFT_REPO_ROOT:-.}"
timeout -k 10 400 python -u -m pytest tests/test_c_perf_gpu.py -x -v --timeout 240 --timeout-method thread > gpurun_out/cperf_tests.log 2>&1 || exit $?
for m in 1 16; do timeout -k 10 120 ./neuronabox-nccl_amd/lib/nbx_perf -c allreduce -d 0,0 -t half -b 4096 -e 4194304 -f 4 -n 20 -w 3 -m $m >> gpurun_out/cperf_agg.txt 2>&1 || exit $?; done
