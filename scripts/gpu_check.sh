#!/usr/bin/env bash
# One GPU-box session: parity tests, smoke, bench, rocprofv3 kernel trace and
# PMC passes. Every GPU step has its own time limit; the script stops at the
# first fault / abort / timeout (exit codes other than 0 or a plain test
# failure) and starts nothing more on the GPU.
set -u
ROOT="${GRAFT_REPO_ROOT:-$(pwd)}"
OUT="$ROOT/gpurun_out/${TAG:-r1}"
mkdir -p "$OUT"
cd "$ROOT"
stop_if_fatal() {   # $1 = rc, $2 = step
  local rc=$1
  echo "[$2] rc=$rc" | tee -a "$OUT/steps.log"
  if [ "$rc" -ne 0 ] && [ "$rc" -ne 1 ]; then echo "fatal rc=$rc at $2; stopping" | tee -a "$OUT/steps.log"; exit "$rc"; fi
}
rocminfo 2>/dev/null | grep -m2 -E "Marketing|gfx9" > "$OUT/device.txt" || true
nproc > "$OUT/nproc.txt"
if [ "${SKIP_TESTS:-0}" != "1" ]; then
  timeout -k 10 900 python -m pytest tests -m gpu -q --maxfail=25 ${PYTEST_ARGS:-} > "$OUT/pytest_gpu.log" 2>&1
  stop_if_fatal $? pytest_gpu
  timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1
  stop_if_fatal $? smoke
fi
timeout -k 10 600 python bench.py ${BENCH_ARGS:-} > "$OUT/bench.json" 2> "$OUT/bench.err"
stop_if_fatal $? bench
if [ "${REHEARSE:-0}" = "1" ]; then   # N=2 launch path with both ranks on the one GPU
  NBX_BENCH_DEVICE=0 NBX_BENCH_BACKEND=gloo timeout -k 10 300 python -m torch.distributed.run --nnodes=1 \
    --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29555 bench.py --gpus 2 --steps 10 --warmup 2 \
    > "$OUT/bench_n2_shared.json" 2> "$OUT/bench_n2_shared.err"
  stop_if_fatal $? bench_n2_rehearsal
fi
if [ "${SKIP_PROF:-0}" != "1" ]; then
  export TMPDIR=/tmp
  timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof" -o trace -- \
    python3 "$ROOT/bench.py" --steps 20 --warmup 3 --no-cpu-baseline > "$OUT/prof_bench.json" 2> "$OUT/prof.err"
  stop_if_fatal $? rocprof_trace
  timeout -k 10 600 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$OUT/pmc_fetch" -o pmc -- \
    python3 "$ROOT/bench.py" --steps 5 --warmup 1 --no-cpu-baseline > "$OUT/pmc_fetch_bench.json" 2> "$OUT/pmc_fetch.err"
  stop_if_fatal $? pmc_fetch
  timeout -k 10 600 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$OUT/pmc_write" -o pmc -- \
    python3 "$ROOT/bench.py" --steps 5 --warmup 1 --no-cpu-baseline > "$OUT/pmc_write_bench.json" 2> "$OUT/pmc_write.err"
  stop_if_fatal $? pmc_write
fi
python3 "$ROOT/scripts/pmc_traffic.py" "$OUT" "$OUT/summary" > "$OUT/pmc_summary.json" 2>&1 || true
echo done | tee -a "$OUT/steps.log"
