# GPUTEST_r05 test order (the 63 tests before the red one, then the multi-process collectives), three times
mkdir -p gpurun_out/r6ab
for rep in 1 2 3; do
NBX_GPU_TEST_ORDER=files timeout -k 10 520 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu \
  tests/test_bench_rccl_gpu.py tests/test_c_perf_gpu.py tests/test_clique_transport_gpu.py tests/test_config_a.py \
  tests/test_configs_gpu.py tests/test_multiprocess_churn_gpu.py \
  tests/test_multiprocess_gpu.py::test_multiprocess_collectives tests/test_multiprocess_gpu.py::test_multiprocess_grouped_collectives \
  tests/test_multiprocess_gpu.py::test_multiprocess_ring_fifo_reduce_scatter_and_reduce tests/test_multiprocess_gpu.py::test_multiprocess_ll_protocol \
  > gpurun_out/r6ab/pytest_r5order_$rep.log 2>&1
rc=$?; echo "rep $rep rc=$rc"; if [ $rc -ne 0 ]; then exit $rc; fi
done
