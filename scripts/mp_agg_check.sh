#!/usr/bin/env bash
# Multi-process groups: nbx_perf -p 1 with 1 vs 16 operations per ncclGroupStart/End
# (Simple protocol forced), 2 ranks sharing the one GPU; profiles/r1/nbx_perf_mp_agg_*.txt
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export NCCL_PROTO=LL,Simple NBX_TIMEOUT_SEC=60 NBX_BOOTSTRAP_TIMEOUT=60 NBX_LL_MAX_GRID=64
for m in 1 16; do
  timeout -k 10 180 ./neuronabox-nccl_amd/lib/nbx_perf -p 1 -c allreduce -d 0,0 -t float -b 131072 -e 16777216 -f 4 \
    -n 20 -w 3 -m $m >> gpurun_out/mp_agg.txt 2>&1 || exit $?
done
NBX_TRACE=1 timeout -k 10 120 ./neuronabox-nccl_amd/lib/nbx_perf -p 1 -c allreduce -d 0,0 -t float -b 1048576 \
  -e 1048576 -n 1 -w 0 -m 4 > gpurun_out/mp_agg_trace.txt 2>&1 || exit $?
