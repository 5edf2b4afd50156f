# 8-rank clique stress after 2/3/4 in the same process: 24 vs 32 hardware queues, and 8,8,8 at 24
mkdir -p gpurun_out/r6x
export NCCL_DEBUG=WARN
NBX_STRESS_HW_QUEUES=32 timeout -k 10 300 python -u scripts/clique_stress.py 2,3,4,8 2 607 > gpurun_out/r6x/q32_2348.jsonl 2> gpurun_out/r6x/q32_2348.err
rc=$?; echo "q32 2,3,4,8 rc=$rc"; if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 300 python -u scripts/clique_stress.py 8,8,8 2 607 > gpurun_out/r6x/q24_888.jsonl 2> gpurun_out/r6x/q24_888.err
rc=$?; echo "q24 8,8,8 rc=$rc"; exit $rc
