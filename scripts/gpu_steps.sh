#!/usr/bin/env bash
# Run GPU steps given as "name|timeout_s|command" lines on stdin, each under its
# own time limit; a plain failure (rc 1) goes on to the next step, anything
# else (fault, abort, timeout) stops the script: nothing more touches the GPU.
set -u
ROOT="${GRAFT_REPO_ROOT:-$(pwd)}"
OUT="$ROOT/gpurun_out/${TAG:-r2}"
mkdir -p "$OUT"
cd "$ROOT"
export TMPDIR=/tmp
while IFS='|' read -r name tmo cmd; do
  [ -z "$name" ] && continue
  echo "[$(date +%T)] start $name" | tee -a "$OUT/steps.log"
  timeout -k 10 "$tmo" bash -c "$cmd" > "$OUT/$name.log" 2>&1
  rc=$?
  echo "[$(date +%T)] $name rc=$rc" | tee -a "$OUT/steps.log"
  if [ "$rc" -ne 0 ] && [ "$rc" -ne 1 ]; then echo "fatal rc=$rc at $name; stopping" | tee -a "$OUT/steps.log"; exit "$rc"; fi
done
echo done | tee -a "$OUT/steps.log"
