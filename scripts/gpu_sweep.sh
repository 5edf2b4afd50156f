#!/usr/bin/env bash
# GPU session: parity tests + bench + library sweeps (see scripts/sweep_lib.py).
set -u
ROOT="${GRAFT_REPO_ROOT:-$(pwd)}"
OUT="$ROOT/gpurun_out/${TAG:-sweep}"
mkdir -p "$OUT"; cd "$ROOT"
fatal() { local rc=$1; echo "[$2] rc=$rc" >> "$OUT/steps.log"; if [ "$rc" -ne 0 ] && [ "$rc" -ne 1 ]; then echo "fatal at $2" >> "$OUT/steps.log"; exit "$rc"; fi; }
if [ "${SKIP_TESTS:-0}" != "1" ]; then
  timeout -k 10 900 python -m pytest tests -m gpu -q --maxfail=25 > "$OUT/pytest_gpu.log" 2>&1; fatal $? pytest
fi
timeout -k 10 600 python bench.py ${BENCH_ARGS:-} > "$OUT/bench.json" 2> "$OUT/bench.err"; fatal $? bench
timeout -k 10 900 python scripts/sweep_lib.py ${SWEEP_ARGS:-} > "$OUT/sweep_lib.jsonl" 2> "$OUT/sweep_lib.err"; fatal $? sweep
echo done >> "$OUT/steps.log"
