# randomized multi-process stress at 8 ranks, six seeds x 40 plans, slice checksums on for odd seeds
mkdir -p gpurun_out/r6aa
for seed in 611 612 613 614 615 616; do
  if [ $((seed % 2)) -eq 1 ]; then chk=1; else chk=0; fi
  NBX_CHECK_SLICES=$chk timeout -k 10 280 python -u scripts/mp_stress.py 8 40 $seed \
    >> gpurun_out/r6aa/mp_stress_8.jsonl 2>> gpurun_out/r6aa/mp_stress_8.err
  rc=$?; echo "seed $seed slices=$chk rc=$rc"; if [ $rc -ne 0 ]; then exit $rc; fi
done
