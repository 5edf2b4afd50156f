# clique stress at 8 ranks (in-kernel transport forced), without and with slice checksums,
# device wait reports on (NCCL_DEBUG=WARN)
mkdir -p gpurun_out/r6v
export NCCL_DEBUG=WARN
timeout -k 10 300 python -u scripts/clique_stress.py 8 3 607 > gpurun_out/r6v/clique8_plain.jsonl 2> gpurun_out/r6v/clique8_plain.err
rc=$?; echo "plain rc=$rc"; if [ $rc -ne 0 ]; then exit $rc; fi
NBX_CHECK_SLICES=1 timeout -k 10 300 python -u scripts/clique_stress.py 8 3 607 > gpurun_out/r6v/clique8_slices.jsonl 2> gpurun_out/r6v/clique8_slices.err
rc=$?; echo "slices rc=$rc"; exit $rc
