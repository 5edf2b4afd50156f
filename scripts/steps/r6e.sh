# round 6: bench + N = 2 rehearsal (mixed_seq leg) + rocprofv3 trace + PMC passes, then the
# mixed-sequence replay with guarded buffers on the default protocols and with the multi-GPU
# protocol gate (LL128 off: every 256 KiB - 1 MiB call takes Simple)
set -u
TAG=r6e REHEARSE=1 SKIP_TESTS=1 bash scripts/gpu_check.sh || exit $?
mkdir -p gpurun_out/r6e
timeout -k 10 300 python -u scripts/mixed_seq_repro.py --ranks 8 --iters 20 --guard --jitter \
  > gpurun_out/r6e/repro_guard.json 2> gpurun_out/r6e/repro_guard.err
rc=$?; echo "repro guard rc=$rc"; if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
NBX_DEBUG_ASSUME_MULTI_GPU=1 timeout -k 10 300 python -u scripts/mixed_seq_repro.py --ranks 8 --iters 20 --guard --jitter \
  > gpurun_out/r6e/repro_gate.json 2> gpurun_out/r6e/repro_gate.err
rc=$?; echo "repro gate rc=$rc"
