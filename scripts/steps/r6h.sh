# round 6: Simple slice checksums (NBX_CHECK_SLICES) on the GPU — the new tests, the mixed
# sequence with the checks on, and the cost: nbx_perf old library (lib_prev: before the
# checksum code) vs new (checks off / on), alternating, NCCL_PROTO=Simple
set -u
OUT=gpurun_out/r6h; mkdir -p $OUT
timeout -k 10 400 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_multiprocess_gpu.py \
  -k "slice_checksum" > $OUT/pytest_slices.log 2>&1
rc=$?; echo "pytest slices rc=$rc"; if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
for rep in 1 2; do
  for lib in prev new newchk; do
    for d in 0,0 0,0,0,0; do
      bin=neuronabox-nccl_amd/lib/nbx_perf; chk=0
      [ $lib = prev ] && bin=neuronabox-nccl_amd/lib_prev/nbx_perf
      [ $lib = newchk ] && chk=1
      NCCL_PROTO=Simple NBX_CHECK_SLICES=$chk timeout -k 10 120 $bin -p 1 -d $d -b 4096 -e 268435456 -f 4 -n 20 -w 5 \
        > $OUT/nbx_perf_${lib}_d${d//,/}_rep$rep.txt 2>&1
      rc=$?; echo "nbx_perf $lib $d rep $rep rc=$rc"; if [ $rc -ne 0 ]; then exit $rc; fi
    done
  done
done
