# the full GPU suite twice on one box (flake hunt: any wrong output describes itself)
mkdir -p gpurun_out/r6o
for rep in 1 2; do
  timeout -k 10 560 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread \
    > gpurun_out/r6o/pytest_gpu_$rep.log 2>&1
  rc=$?; echo "rep $rep rc=$rc"; if [ $rc -ne 0 ]; then exit $rc; fi
done
