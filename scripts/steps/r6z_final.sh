# final tree: the GPU suite as the driver runs it, smoke, bench
mkdir -p gpurun_out/r6z
timeout -k 10 700 python -u -m pytest tests/ -x -q -m gpu > gpurun_out/r6z/pytest_gpu.log 2>&1
rc=$?; echo "suite rc=$rc"; if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r6z/smoke.log 2>&1
rc=$?; echo "smoke rc=$rc"; if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 400 python -u bench.py > gpurun_out/r6z/bench.json 2> gpurun_out/r6z/bench.err
rc=$?; echo "bench rc=$rc"; exit $rc
