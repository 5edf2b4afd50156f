# the GPU suite exactly as the round-end driver runs it (-x -q, no per-test timeout),
# once in the suite's order and once in plain collection order (GPUTEST_r05's order)
mkdir -p gpurun_out/r6s
timeout -k 10 560 python -u -m pytest tests/ -x -q -m gpu > gpurun_out/r6s/pytest_gpu_driver_style.log 2>&1
rc=$?; echo "suite order rc=$rc"; if [ $rc -ne 0 ]; then exit $rc; fi
NBX_GPU_TEST_ORDER=files timeout -k 10 560 python -u -m pytest tests/ -x -q -m gpu \
  > gpurun_out/r6s/pytest_gpu_driver_style_files_order.log 2>&1
rc=$?; echo "collection order rc=$rc"; exit $rc
