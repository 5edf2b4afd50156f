#!/usr/bin/env python3
"""bench.py — BASELINE metric: GiB/s of the device-resident ncclSum reduction.

Workload (BASELINE.json configs[1]): one step = one
call of the hot path, nbxReduceMulti (the reduceCopy replacement), folding
8 fp32 inputs of 256 MiB (67,108,864 elements) into one 256 MiB output on the
GPU — 2.25 GiB of algorithmic HBM traffic per step, inputs resident in HBM
before timing starts.

N GPUs (one process per GPU, torch.distributed.run): every rank reduces its
own 8 x 256 MiB shard (the path shards by chunk; no data-path collective), so
scaling is weak and value = N x 2.25 GiB / max-over-ranks step time.

Extra JSON fields:
  roofline     — the dominant kernel's algorithmic bytes per launch / its mean
                 launch duration (HIP events on the launch stream) vs the
                 8 TB/s HBM3E peak; `traffic` = HBM bytes per launch from the
                 committed rocprofv3 PMC pass (profiles/pmc_latest.json) — NOT
                 measured in this run: `traffic_provenance` names its box/run;
                 `ceiling_mixed` = the same tile's 8:1 read/write stream with
                 no arithmetic, measured here, and frac_of_ceiling = achieved /
                 ceiling_mixed.
  cpu_baseline — the oracle's C restatement (oracle/reduce_oracle.c, a port of
                 the reference semantics) timed on this box's host cores on a
                 bounded sample of the same workload (rank 0, N=1 only).
  collective   — N > 1 only, after the timed region: SURVEY §8(d) config D
                 (ncclAllReduce direct + ring, ncclReduceScatter, 1 GiB fp32
                 per rank, and a 4 KiB LL AllReduce) through libnbxccl's
                 multi-process communicator across the N GPUs, checked exactly;
                 run in a child process per rank (scripts/collective_leg.py) so
                 a failure there is reported here instead of ending the bench.
                 Then `collective.clique`: config D through the single-process
                 communicator (ncclCommInitAll over the same N GPUs, no IPC;
                 scripts/clique_leg.py, a child of rank 0), so a multi-process
                 plumbing failure can be told from an xGMI data-path failure.
                 Then `collective.rccl`: RCCL (torch.distributed "nccl") on the
                 same shapes in the bench process, as the vendor reference.
                 NBX_BENCH_COLLECTIVE=0 skips all three, NBX_BENCH_CLIQUE=0 the
                 clique part, NBX_BENCH_RCCL=0 the RCCL part.

The N > 1 legs share ONE wall budget, NBX_BENCH_LEG_BUDGET_S (default 240 s,
so an 8-rank run stays well inside a 600 s driver limit): every leg's wait is
drawn from what is left of it (rank 0's clock, broadcast, so every rank makes
the same skip decision), a leg that no longer fits is skipped with the reason
recorded, a leg that times out reports the last partial result its child
printed, and a watchdog ends every rank at the budget (+ a grace) even if a
leg hangs inside this process (RCCL). At N > 1 rank 0 prints the headline line
(value, roofline) BEFORE the legs start and again, with `collective` filled
in, when they end (or when the watchdog fires): a stall in never-on-xGMI code
can cost the collective evidence, never the headline value.
"""
from __future__ import annotations

import argparse
import json
import os
import select
import subprocess
import sys
import tempfile
import threading
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)

COLLECTIVE_SCRIPT = os.path.join(ROOT, "scripts", "collective_leg.py")
CLIQUE_SCRIPT = os.path.join(ROOT, "scripts", "clique_leg.py")
LEG_BUDGET_S = 240.0     # NBX_BENCH_LEG_BUDGET_S: every N > 1 leg together
# a leg is skipped when less than this is left (and each leg keeps this much
# for every leg after it); the watchdog fires this long after the budget
LEG_MIN_S = float(os.environ.get("NBX_BENCH_LEG_MIN_S", "15"))
WATCHDOG_GRACE_S = float(os.environ.get("NBX_BENCH_WATCHDOG_GRACE_S", "20"))

N_SRCS = 8
COUNT = 64 << 20                    # fp32 elements per 256 MiB input
ELT = 4
ALG_BYTES = (N_SRCS + 1) * COUNT * ELT   # (nSrcs + nDsts) x count x sizeof(T), SURVEY §8(d)
HBM_PEAK_GBS = 8000.0               # MI355X HBM3E spec peak, MI355X_MICROARCH.md
METRIC = "GiB/s device-resident ncclSum reduce, 256 MiB fp32, 1/2/4/8 MI355X (% HBM peak)"


def _load_package():
    from __graft_entry__ import _load_package as lp
    return lp()


def _build_stamp(nbx) -> dict:
    """Which build of libnbxccl.so produced the line (the stamp build() wrote,
    neuronabox-nccl_amd/lib/build_info.json) and whether the library and the
    sources on this box are still that build."""
    bi = nbx.build_info()
    rec = bi["recorded"] or {}
    return {"sources_sha256": rec.get("sources_sha256"), "lib_sha256": rec.get("lib_sha256"),
            "lib_matches": bi["lib_matches"], "sources_match": bi["sources_match"]}


def _dist_init():
    """One process per GPU (torch.distributed.run env). The process group is the
    control plane only (barrier + max-over-ranks): RCCL ("nccl") by default,
    NBX_BENCH_BACKEND=gloo to keep it on the CPU. NBX_BENCH_DEVICE pins every
    rank to one device (rehearsing N > 1 on a one-GPU box)."""
    import torch
    import torch.distributed as dist
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    dev = int(os.environ.get("NBX_BENCH_DEVICE", local))
    if torch.cuda.is_available():
        torch.cuda.set_device(dev)
    if world > 1:
        backend = os.environ.get("NBX_BENCH_BACKEND") or ("nccl" if torch.cuda.is_available() else "gloo")
        init_process_group(backend, rank, world, dev)
    return world, rank, dev


def init_process_group(backend: str, rank: int, world: int, dev: int):
    """The bench's process group (tests/test_bench_rccl_gpu.py runs this with
    backend "nccl" at one rank, so the RCCL path is exercised before the
    driver's multi-GPU run)."""
    import torch
    import torch.distributed as dist
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    dist.init_process_group(backend=backend, rank=rank, world_size=world,
                            device_id=torch.device("cuda", dev) if backend == "nccl" else None)


def _barrier(world):
    if world > 1:
        import torch.distributed as dist
        dist.barrier()


def max_over_ranks(value: float, world: int) -> float:
    """Max of a host float over ranks (the contract's max-over-ranks timing);
    through the process group whenever one exists (also at one rank)."""
    import torch.distributed as dist
    if world == 1 and not (dist.is_available() and dist.is_initialized()):
        return value
    import torch
    dev = torch.device("cuda", torch.cuda.current_device()) if dist.get_backend() == "nccl" else "cpu"
    t = torch.tensor([value], dtype=torch.float64, device=dev)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


class LegBudget:
    """One wall budget shared by every N > 1 leg (NBX_BENCH_LEG_BUDGET_S)."""

    def __init__(self, total: float | None = None, clock=time.monotonic):
        if total is None:
            total = float(os.environ.get("NBX_BENCH_LEG_BUDGET_S", LEG_BUDGET_S))
        self.total = float(total)
        self.clock = clock
        self.t0 = clock()

    def left(self) -> float:
        return max(0.0, self.total - (self.clock() - self.t0))

    def agreed_left(self, world: int) -> float:
        """Rank 0's remaining budget, the same on every rank (one broadcast):
        every rank then skips, or bounds, a leg alike."""
        left = self.left()
        if world > 1:
            import torch.distributed as dist
            if dist.is_available() and dist.is_initialized():
                box = [left]
                dist.broadcast_object_list(box, src=0)
                left = float(box[0])
        return left


def leg_timeout(default: float, left: float, reserve: float = 0.0) -> float:
    """A leg's wait: its own default, capped by what is left of the budget
    after `reserve` seconds kept for the legs that follow it."""
    return max(0.0, min(default, left - reserve))


def skipped_leg(left: float, what: str) -> dict:
    return {"ok": False, "skipped": f"{what} skipped: {left:.0f} s of the leg budget left "
                                    f"(NBX_BENCH_LEG_BUDGET_S), under the {LEG_MIN_S:.0f} s minimum"}


class Emitter:
    """Rank 0's JSON lines. The final line is printed once, by the main
    thread when the legs end or by the watchdog when the budget runs out."""

    def __init__(self, rank: int):
        self.rank = rank
        self.lock = threading.Lock()
        self.final_done = False
        self.result = None      # the headline result, once measured
        self.coll = None        # the collective summary built so far
        self.leg = None         # the leg running now (for the watchdog's reason)

    def preliminary(self, result: dict) -> None:
        if self.rank != 0:
            return
        line = dict(result)
        line["collective"] = {"ok": None, "status": "pending: the N > 1 legs run after this line; "
                                                    "the final line (same value) follows"}
        with self.lock:
            print(json.dumps(line), flush=True)

    def final(self, result: dict, reason: str | None = None) -> None:
        with self.lock:
            if self.final_done:
                return
            self.final_done = True
            if self.rank != 0:
                return
            line = dict(result)
            if reason is not None:
                coll = dict(self.coll or {})
                coll["ok"] = False
                coll.setdefault("errors", []).append(reason)
                coll["incomplete"] = reason
                line["collective"] = coll
            print(json.dumps(line), flush=True)


# Exit status of a run whose N > 1 legs were cut off (a leg gave no result in
# its time, or the watchdog ended the run): the final line is printed first and
# keeps the headline value, but the status tells a harness that checks it
# that a leg hung. A complete run exits 0.
EXIT_LEG_CUT_OFF = 3


def legs_cut_off(coll) -> bool:
    """True when any N > 1 leg of the final line ended without its result."""
    if not isinstance(coll, dict):
        return False
    if coll.get("incomplete"):
        return True
    return any(isinstance(v, dict) and v.get("incomplete") for v in coll.values())


class Watchdog:
    """Ends this rank when the leg budget (+ grace) is spent: rank 0 prints the
    final line with what the legs produced so far and the reason, every rank
    kills its own leg children (by PID) and exits EXIT_LEG_CUT_OFF — the
    headline value stands in the line; `collective.ok` is false."""

    def __init__(self, seconds: float, emitter: Emitter, children, exit_fn=None):
        self.emitter = emitter
        self.children = [c for c in children if c is not None]
        self.exit_fn = exit_fn or (lambda: os._exit(EXIT_LEG_CUT_OFF))
        self.cancelled = threading.Event()
        self.seconds = seconds
        self.thread = threading.Thread(target=self._run, daemon=True)
        self.thread.start()

    def _run(self):
        if self.cancelled.wait(self.seconds):
            return
        leg = self.emitter.leg or "the legs"
        print(f"[bench rank {self.emitter.rank}] leg budget spent during {leg}; ending the run", file=sys.stderr,
              flush=True)
        if self.emitter.result is not None:
            self.emitter.final(self.emitter.result,
                               f"leg budget ({self.seconds:.0f} s incl. grace) spent during {leg}; "
                               "the run was ended by the watchdog")
        for c in self.children:
            try:
                c.kill()   # this rank's own child, by PID
            except OSError:
                pass
        sys.stdout.flush()
        sys.stderr.flush()
        self.exit_fn()

    def cancel(self):
        self.cancelled.set()


def _pmc_traffic():
    """(HBM bytes per launch, provenance) of the f32 sum 8-src kernel from the
    committed PMC summary (profiles/pmc_latest.json, written by
    scripts/pmc_traffic.py from separate rocprofv3 --pmc passes, FETCH_SIZE
    doubled per the gfx950 note). Carried over from that run, not measured by
    this bench invocation; the provenance string says so."""
    p = os.path.join(ROOT, "profiles", "pmc_latest.json")
    try:
        with open(p) as f:
            d = json.load(f)
        if d.get("workload") == "config_b_f32_sum_8x256MiB":
            src = d.get("source", "")
            return d.get("hbm_bytes_per_launch"), (
                f"carried over from profiles/pmc_latest.json ({src or 'committed rocprofv3 --pmc passes'}); "
                "not measured in this run")
    except (OSError, ValueError):
        pass
    return None, None


def host_e2e_leg(torch, nbx, srcs, out, stream, op, reps: int = 2):
    """BASELINE: the path starts and ends in host memory. Config B with the
    8 inputs and the output in pinned host memory: nbxReduceMultiHost
    (zero-copy: the kernel reads / writes the pinned buffers over PCIe) and
    the naive H2D -> reduce -> D2H sequence. PCIe-inclusive; never `value`."""
    f32 = int(nbx.ncclDataType.ncclFloat32)
    hs = [s.cpu().pin_memory() for s in srcs]   # the same seeded inputs
    ho = torch.empty(COUNT, dtype=torch.float32).pin_memory()
    sh = stream.cuda_stream
    hp = [h.data_ptr() for h in hs]
    nbx.reduce_multi_host([ho.data_ptr()], hp, COUNT, f32, op, 0, False, sh)   # warm
    t0 = time.perf_counter()
    for _ in range(reps):
        nbx.reduce_multi_host([ho.data_ptr()], hp, COUNT, f32, op, 0, False, sh)
    zms = (time.perf_counter() - t0) * 1e3 / reps
    ok = bool(torch.equal(ho[:1 << 16], out[:1 << 16].cpu()))
    dptr = [s.data_ptr() for s in srcs]
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(reps):
        for h, d in zip(hs, srcs):
            d.copy_(h, non_blocking=True)
        nbx.reduce_multi([out.data_ptr()], dptr, COUNT, f32, op, 0, False, sh)
        ho.copy_(out, non_blocking=True)
        torch.cuda.synchronize()
    nms = (time.perf_counter() - t0) * 1e3 / reps
    return {"what": "config B with inputs and output in pinned host memory (PCIe-inclusive; not `value`)",
            "zero_copy_ms": round(zms, 3), "zero_copy_GiBps": round(ALG_BYTES / (zms * 1e-3) / 2**30, 2),
            "naive_h2d_reduce_d2h_ms": round(nms, 3),
            "naive_GiBps": round(ALG_BYTES / (nms * 1e-3) / 2**30, 2), "matches_device_result": ok}


def host_cpu_share():
    """(threads this process may run in parallel, CPUs on the box): the
    affinity mask, capped by the cgroup CPU quota when there is one (the GPU
    box grants each GPU's jobs a share of the host's CPUs)."""
    on_box = os.cpu_count() or 1
    try:
        aff = len(os.sched_getaffinity(0))
    except (AttributeError, OSError):
        aff = on_box
    quota = None
    try:
        with open("/sys/fs/cgroup/cpu.max") as f:
            q, period = f.read().split()[:2]
            if q != "max":
                quota = max(1, int(int(q) / int(period)))
    except (OSError, ValueError):
        pass
    return (min(aff, quota) if quota else aff), on_box, quota


def stream_ceilings(torch, nbx, srcs, out, stream, reps: int = 10):
    """HBM stream ceilings on THIS box, same process, right after the timed
    region: read-only over the config-B inputs with the hot
    kernel's loads and tile, write-only with its stores, and a 1:1 copy
    (the production kernel at one source) of the config-B byte count."""
    import ctypes
    lib = nbx.load_library()
    lib.nbxDebugStream.argtypes = [ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int, ctypes.c_size_t,
                                   ctypes.c_int, ctypes.c_void_p]
    sh = ctypes.c_void_p(stream.cuda_stream)
    half = ALG_BYTES // 2   # copy: read + write = the config-B byte count
    a = torch.empty(half // 4, dtype=torch.float32, device=out.device).uniform_(-1, 1)
    b = torch.empty_like(a)
    s_arr = (ctypes.c_void_p * N_SRCS)(*[t.data_ptr() for t in srcs])
    f32 = int(nbx.ncclDataType.ncclFloat32)
    op = nbx.host_to_dev_redop(nbx.ncclRedOp.ncclSum, nbx.ncclDataType.ncclFloat32, 1)
    a_arr = (ctypes.c_void_p * 1)(a.data_ptr())
    b_arr = (ctypes.c_void_p * 1)(b.data_ptr())

    def timed(fn, nbytes):
        for _ in range(2):
            fn()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(stream)
        for _ in range(reps):
            fn()
        e1.record(stream)
        torch.cuda.synchronize()
        return round(nbytes / (e0.elapsed_time(e1) / reps * 1e-3) / 1e9, 1)

    def chk(rc):
        if rc != 0:
            raise RuntimeError(f"stream ceiling launch failed: {rc}")
    rd = timed(lambda: chk(lib.nbxDebugStream(0, out.data_ptr(), s_arr, N_SRCS, COUNT * ELT, 0, sh)),
               N_SRCS * COUNT * ELT)
    mx = timed(lambda: chk(lib.nbxDebugStream(2, b.data_ptr(), s_arr, N_SRCS, COUNT * ELT, 0, sh)), ALG_BYTES)
    wr = timed(lambda: chk(lib.nbxDebugStream(1, b.data_ptr(), None, 0, half, 0, sh)), half)
    cp = timed(lambda: chk(lib.nbxReduceMulti(b_arr, 1, a_arr, 1, half // 4, f32, op, 0, 0, sh)), 2 * half)
    del a, b
    return {"read_GBs": rd, "write_GBs": wr, "copy_GBs": cp, "mixed_GBs": mx,
            "what": "same process, this box: read-only 8 x 256 MiB (hot kernel's nt loads, 8x4 packs/lane, "
                    "1 WG/CU, nothing stored); write-only 1.125 GiB (plain 16-B stores); 1:1 copy 1.125 GiB -> "
                    "1.125 GiB (nbxReduceMulti, 1 source); mixed 8:1 = the hot kernel's tile and schedule reading "
                    "8 x 256 MiB and storing 256 MiB with no arithmetic"}


def cpu_baseline(seconds: float = 1.5):
    """Oracle (C port of the reference semantics) on host cores, same workload
    shape, bounded sample: passes over the full config-B workload for about
    `seconds` of wall time; `value` is the best pass (BASELINE.md's CPU plan:
    best of the runs), the mean is in `sample`. Also config A (2 x 4 MiB fp32,
    the reference's CPU-runnable case), best of 5. Returns the cpu_baseline
    JSON object."""
    import numpy as np
    from oracle import oracle   # checker / baseline only
    oracle.build()
    share, on_box, quota = host_cpu_share()
    threads = int(os.environ.get("NBX_CPU_THREADS", "0")) or share
    rng = np.random.default_rng(1234)
    srcs = [rng.uniform(-1, 1, COUNT).astype(np.float32) for _ in range(N_SRCS)]
    out = [np.empty(COUNT, np.float32)]
    oracle.reduce_multi(srcs, 7, 0, threads=threads, out=out)   # warm (page-in)
    t0 = time.perf_counter()
    passes = []
    while True:
        t1 = time.perf_counter()
        oracle.reduce_multi(srcs, 7, 0, threads=threads, out=out)
        passes.append(time.perf_counter() - t1)
        el = time.perf_counter() - t0
        if el >= seconds and len(passes) >= 5:
            break
    best, mean = min(passes), sum(passes) / len(passes)
    del srcs, out
    a = oracle.random_inputs(7, 2, 1 << 20, seed=1234)   # config A
    oa = [np.empty(1 << 20, np.float32)]
    ta = []
    for _ in range(6):
        t1 = time.perf_counter()
        oracle.reduce_multi(a, 7, 0, threads=threads, out=oa)
        ta.append(time.perf_counter() - t1)
    ta = min(ta[1:])
    return {"value": round(ALG_BYTES / best / 2**30, 3), "unit": "GiB/s", "cores": threads, "kind": "port",
            "cores_used": threads, "cores_on_box": on_box, "cpu_quota": quota,
            "sample": f"{len(passes)} passes of the full config-B workload (8 x 256 MiB fp32 -> 256 MiB), "
                      f"{el:.2f} s wall x {threads} threads, oracle/reduce_oracle.c (gcc -O3); value = best pass, "
                      f"mean {ALG_BYTES / mean / 2**30:.1f} GiB/s",
            "config_a": {"value": round(3 * (1 << 20) * 4 / ta / 2**30, 3), "unit": "GiB/s", "ms": round(ta * 1e3, 4),
                         "what": "2 x 4 MiB fp32 sum (BASELINE config A), best of 5, same threads"}}


def _spawn_collective_leg(world: int, script: str | None = None):
    """Start this rank's collective-leg child before the parent touches the GPU."""
    if world <= 1 or os.environ.get("NBX_BENCH_COLLECTIVE", "1") == "0":
        return None
    script = script or COLLECTIVE_SCRIPT
    log = tempfile.NamedTemporaryFile(prefix=f"nbx_coll_leg_r{os.environ.get('RANK', '0')}_", suffix=".log",
                                      delete=False)
    child = subprocess.Popen([sys.executable, script],
                             stdin=subprocess.PIPE, stdout=subprocess.PIPE, stderr=log, text=True, bufsize=1,
                             cwd=ROOT)
    child.nbx_log = log.name
    return child


def _spawn_clique_leg(world: int, rank: int, script: str | None = None):
    """Rank 0 only: start the single-process clique child before the parent
    touches the GPU; it stays idle (no HIP call) until told to run."""
    if (world <= 1 or rank != 0 or os.environ.get("NBX_BENCH_COLLECTIVE", "1") == "0"
            or os.environ.get("NBX_BENCH_CLIQUE", "1") == "0"):
        return None
    return _spawn_collective_leg(world, script or CLIQUE_SCRIPT)


def _close_child(child):
    if child is None:
        return
    try:
        child.stdin.close()
    except OSError:
        pass
    try:
        child.wait(timeout=5)
    except subprocess.TimeoutExpired:
        child.kill()   # this rank's own child, by PID
        child.wait()


def clique_leg(child, world: int, rank: int, dev: int, result_timeout: float = 400.0,
               budget: LegBudget | None = None):
    """Config D through ncclCommInitAll over every rank's GPU, run by rank 0's
    child while the other ranks wait on the host (the process group's store:
    no RCCL kernel of theirs occupies a GPU meanwhile). Rank 0 gets the result.
    With a budget the wait is capped by what is left of it (rank 0's clock)."""
    import datetime
    import torch.distributed as dist
    if budget is not None:
        left = budget.agreed_left(world)
        if left < LEG_MIN_S:
            if rank == 0:
                _close_child(child)
                return skipped_leg(left, "the clique leg")
            return None
        result_timeout = leg_timeout(result_timeout, left, reserve=LEG_MIN_S)
    devs = [None] * world
    dist.all_gather_object(devs, dev)
    store = dist.distributed_c10d._get_default_store()
    key = "nbx_clique_leg_done"
    if rank != 0:
        try:
            store.wait([key], datetime.timedelta(seconds=result_timeout + 10))
        except Exception as e:   # rank 0 never set the key: its wait is bounded too; go on
            print(f"[bench rank {rank}] clique leg: no completion from rank 0 ({type(e).__name__})",
                  file=sys.stderr, flush=True)
        return None
    res = None
    partial = None
    if child is not None:
        try:
            child.stdin.write(f"RUN {world} {','.join(str(d) for d in devs)}\n")
            child.stdin.flush()
            line, partial = _read_line(child, "RESULT", result_timeout, partial=True)
            res = json.loads(line) if line else None
        except (OSError, ValueError):
            res = None
        try:
            child.stdin.close()
        except OSError:
            pass
        try:
            child.wait(timeout=60 if res is not None else 1)
        except subprocess.TimeoutExpired:
            child.kill()   # rank 0's own child, by PID
            child.wait()
        if res is None:
            res = _partial_or_error(partial, f"no result from the clique leg within {result_timeout:.0f} s: "
                                    + _log_tail(child))
    store.set(key, "1")
    if res is None:
        return None
    S = COUNT_D * 4
    for name, fac in (("allreduce", 2 * (world - 1) / world), ("reduce_scatter", (world - 1) / world),
                      ("fold_allreduce", 2 * (world - 1) / world), ("fold_reduce_scatter", (world - 1) / world)):
        ms = res.get(name + "_ms")
        if ms:
            alg = S / (ms * 1e-3) / 1e9
            res[name] = {"ms": round(ms, 4), "algbw_GBs": round(alg, 2), "busbw_GBs": round(alg * fac, 2)}
    n, M = world, S
    # local HBM rate per GPU: in-kernel entries on the staging
    # model of the multi-process kernels (same kernels); the direct fold reads
    # every rank's block in place (M) and writes its block into every output
    # (M) / its own output (M / n) — model bytes, no PMC ratio measured
    # (without the in-kernel transport — ranks sharing a GPU — `allreduce` /
    # `reduce_scatter` ran on the fold too: `simple_in_kernel` false)
    ik = res.get("simple_in_kernel", True) is not False
    for name, model in (("allreduce", 2 * (M + 2 * (n - 1) * M // n) if ik else 2 * M),
                        ("reduce_scatter", 2 * (n - 1) * M // n + M + M // n if ik else M + M // n),
                        ("fold_allreduce", 2 * M), ("fold_reduce_scatter", M + M // n)):
        e = res.get(name)
        if isinstance(e, dict) and e.get("ms"):
            e["hbm_model_bytes_per_rank"] = model
            e["hbm_GBs_per_rank"] = round(model / (e["ms"] * 1e-3) / 1e9, 1)
    res["workload"] = ("config D through ncclCommInitAll (one process, every GPU of the run, no IPC), "
                       "ncclSum fp32 1 GiB per rank, checked exactly; allreduce / reduce_scatter on the in-kernel Simple transport over staging "
                       "(forced for every size), fold_* on the event-ordered direct fold (NBX_CLIQUE_SIMPLE=0; the "
                       "clique's default above NBX_CLIQUE_SIMPLE_MAX_BYTES = 32 MiB)")
    return res


def _read_line(child, prefix: str, timeout: float, partial: bool = False):
    """Next line of the child's stdout starting with `prefix`; a heartbeat goes
    to stderr every 30 s while waiting (a long leg never looks hung). With
    `partial`, returns (line, last PARTIAL json the child printed meanwhile):
    the legs print their results so far after every stage."""
    deadline = time.monotonic() + timeout
    t0 = time.monotonic()
    last = None
    found = None
    while time.monotonic() < deadline:
        r, _, _ = select.select([child.stdout], [], [], max(0.0, min(30.0, deadline - time.monotonic())))
        if not r:
            if time.monotonic() < deadline:
                print(f"[bench rank {os.environ.get('RANK', '0')}] collective leg running "
                      f"({time.monotonic() - t0:.0f} s)", file=sys.stderr, flush=True)
                continue
            break
        line = child.stdout.readline()
        if not line:
            break   # child exited
        if line.startswith("PARTIAL "):
            try:
                last = json.loads(line[len("PARTIAL "):])
            except ValueError:
                pass
            continue
        if line.startswith(prefix + " "):
            found = line[len(prefix) + 1:].strip()
            break
    return (found, last) if partial else found


def _partial_or_error(partial, reason: str) -> dict:
    """A leg that gave no final result: its last partial result (if any),
    marked failed, with the reason."""
    res = dict(partial) if isinstance(partial, dict) else {}
    res["ok"] = False
    res["errors"] = list(res.get("errors") or []) + [reason]
    res["incomplete"] = True
    return res


def _log_tail(child, n=5):
    try:
        with open(child.nbx_log) as f:
            return " | ".join(f.read().strip().splitlines()[-n:])
    except OSError:
        return ""


def collective_leg(child, world: int, rank: int, result_timeout: float = 400.0, budget: LegBudget | None = None,
                   reserve: float = 0.0):
    """Drive the child through config D; every rank returns; rank 0 gets the
    summary. With a budget, the ID handshake and the run wait at most what is
    left of it (rank 0's clock) minus `reserve` for the legs after this one."""
    import torch.distributed as dist
    id_timeout = 180.0
    if budget is not None:
        left = budget.agreed_left(world)
        if left - reserve < LEG_MIN_S:
            _close_child(child)
            return skipped_leg(left, "the collective leg") if rank == 0 else None
        id_timeout = leg_timeout(id_timeout, left, reserve=reserve + LEG_MIN_S)
    ids = None
    if rank == 0:
        try:
            child.stdin.write("ID\n")
            child.stdin.flush()
            ids = _read_line(child, "ID", id_timeout)
        except OSError:
            ids = None
    box = [ids]
    dist.broadcast_object_list(box, src=0)
    ids = box[0]
    if budget is not None:
        result_timeout = leg_timeout(result_timeout, budget.agreed_left(world), reserve=reserve)
    res = None
    partial = None
    if ids is not None:
        try:
            child.stdin.write(f"RUN {ids}\n")
            child.stdin.flush()
            line, partial = _read_line(child, "RESULT", result_timeout, partial=True)
            res = json.loads(line) if line else None
        except (OSError, ValueError):
            res = None
    got = res is not None
    try:
        child.stdin.close()
    except OSError:
        pass
    try:
        child.wait(timeout=60 if got else 1)
    except subprocess.TimeoutExpired:
        child.kill()   # this rank's own child, by PID
        child.wait()
    if not got:
        why = ("no unique ids from rank 0's collective-leg child" if ids is None else
               f"no result from the collective leg within {result_timeout:.0f} s")
        res = _partial_or_error(partial, why + ": " + _log_tail(child))
        res["rank"] = rank
    allres = [None] * world
    dist.all_gather_object(allres, res)
    if rank != 0:
        return None
    S = COUNT_D * 4
    out = {"workload": "config D: 1 GiB fp32 per rank, ncclSum, one process per GPU, libnbxccl multi-process "
                       "communicator (TCP bootstrap, hipIpc peer buffers, device flags)",
           "n_ranks": world, "ok": all(r.get("ok") for r in allres),
           # every rank pinned to one GPU (NBX_BENCH_DEVICE: a rehearsal, not xGMI)
           "shared_gpu": "NBX_BENCH_DEVICE" in os.environ,
           "check": "exact (small-integer fp32 inputs), whole output, every rank"}
    errs = [f"rank {r.get('rank')}: {e}" for r in allres for e in r.get("errors", [])]
    if errs:
        out["errors"] = errs[:8]
    if any(r.get("incomplete") for r in allres):
        out["incomplete"] = True   # a rank's leg gave no final result (exit status EXIT_LEG_CUT_OFF)

    def agg(key, busfac, alg_bytes):
        vals = [r.get(key) for r in allres]
        if any(v is None for v in vals):
            return None
        ms = max(vals)
        alg = alg_bytes / (ms * 1e-3) / 1e9
        return {"ms": round(ms, 4), "algbw_GBs": round(alg, 2), "busbw_GBs": round(alg * busfac, 2)}
    out["allreduce_direct"] = agg("allreduce_direct_ms", 2 * (world - 1) / world, S)
    out["allreduce_ring"] = agg("allreduce_ring_ms", 2 * (world - 1) / world, S)
    out["reduce_scatter"] = agg("reduce_scatter_ms", (world - 1) / world, S)
    E = 128 << 20
    out["config_e"] = {"int64_max": agg("config_e_int64_max_ms", 2 * (world - 1) / world, E),
                       "fp8_e4m3_sum": agg("config_e_fp8_sum_ms", 2 * (world - 1) / world, E),
                       "check": "bit-exact vs a GPU restatement of the direct schedule's fold order"}
    for key in ("ll_allreduce_4KiB_us", "ll128_allreduce_1MiB_us"):
        vals = [r.get(key) for r in allres]
        out[key] = None if any(v is None for v in vals) else round(max(vals), 2)
    sw = {"bytes": allres[0].get("sweep_bytes"), "what": "fp32 sum AllReduce us/call, max over ranks, per protocol"}
    for name in ("LL", "LL128", "LL128_oneshot", "Simple"):
        rows = [r.get("sweep_" + name + "_us") for r in allres]
        sw[name] = None if any(v is None for v in rows) else [max(col) for col in zip(*rows)]
    out["protocol_sweep"] = sw
    # LL128 kept by every rank's creation-time probe (else LL / Simple carried those sizes)
    act = [r.get("ll128_active") for r in allres]
    out["ll128_active"] = None if any(a is None for a in act) else all(act)
    out["hbm_model"] = simple_hbm_model(world, S)
    # LL_CASES back to back on the default protocols, every output exact
    ms = [r.get("mixed_seq_mismatches") for r in allres]
    mc = [r.get("mixed_seq_checked_calls") for r in allres]
    out["mixed_seq"] = None if any(v is None for v in ms + mc) else {
        "checked_calls": sum(mc), "mismatches_per_rank": ms,
        "what": "tests' LL_CASES (LL / LL128 / Simple sizes, misaligned offsets) issued back to back without host "
                "sync, 3 iterations, max / min on full-range values, sums on small integers: exact on the GPU"}
    out["transport_allreduce"] = agg("transport_allreduce_ms", 2 * (world - 1) / world, S)
    add_hbm_rates(out, world, S)
    add_fabric_rates(out, allres, world, S)
    cv = [r.get("curve_allreduce_ms") for r in allres]
    if cv and all(isinstance(c, list) and len(c) == len(CURVE_BYTES) for c in cv):
        out["allreduce_curve"] = {"bytes": list(CURVE_BYTES), "ms": [round(max(col), 4) for col in zip(*cv)],
                                  "busbw_GBs": [round(b / (max(col) * 1e-3) / 1e9 * 2 * (world - 1) / world, 2)
                                                for b, col in zip(CURVE_BYTES, zip(*cv))]}
    # the Simple transport's knobs on the same 1 GiB AllReduce (max over ranks)
    kn = [r.get("simple_knobs_ms") for r in allres]
    if all(isinstance(k, dict) for k in kn) and kn:
        out["simple_knobs"] = {name: round(max(k.get(name, 0.0) for k in kn), 4) for name in kn[0]}
        out["simple_knobs"]["default"] = (out.get("allreduce_direct") or {}).get("ms")
    # LL128 forced across the fabric (NCCL_PROTO=LL128): every call checked
    fc = [r.get("ll128_forced_checked_calls") for r in allres]
    fm = [r.get("ll128_forced_mismatched_calls") for r in allres]
    out["ll128_forced"] = (None if any(v is None for v in fc + fm) else
                           {"checked_calls": sum(fc), "mismatched_calls": sum(fm), "per_rank_mismatched": fm,
                            "what": "AllReduces on the NCCL_PROTO=LL128 communicator, one-shot 96 KiB and (n > 2) "
                                    "two-shot 1 MiB, inputs changing per call, every output compared exactly"})
    # connection buffers re-exported at creation (a wrong IPC mapping, verified before first use)
    rep = [r.get("ipc_repairs") for r in allres]
    out["ipc_repairs"] = (None if any(v is None for v in rep) else
                          {k: sum((v.get(k) or 0) for v in rep) for k in ("direct", "ring")})
    return out


def add_hbm_rates(out: dict, world: int, msg_bytes: int) -> None:
    """the local HBM rate per GPU of each libnbxccl
    entry = the staging design's HBM bytes per rank (simple_hbm_model; for
    ReduceScatter and the transport-only call their own model) x the measured
    HBM / model ratio of the same kernels (committed PMC passes; 1.0 where none
    was measured) / the call's time. A model-derived rate, stated as such."""
    n, M = world, msg_bytes
    hm = out.get("hbm_model") or simple_hbm_model(world, msg_bytes)
    ratio = hm.get("measured_over_model") or {}
    models = {
        # push (n-1) blocks + fold M + store and push the block n times + gather (n-1) blocks
        "allreduce_direct": (2 * (M + 2 * (n - 1) * M // n), "direct"),
        "allreduce_ring": (2 * (M + 2 * (n - 1) * M // n), "ring"),
        # push (n-1) blocks, fold M, store one block
        "reduce_scatter": (2 * (n - 1) * M // n + M + M // n, "direct"),
        # as allreduce_direct without reading the n-1 staging slots of the fold
        "transport_allreduce": (4 * (n - 1) * M // n + M // n + M, None),
    }
    for key, (model, rkey) in models.items():
        e = out.get(key)
        if not e or not e.get("ms"):
            continue
        r = ratio.get(rkey) if rkey else None
        e["hbm_model_bytes_per_rank"] = model
        e["hbm_over_model_applied"] = r if r else 1.0
        e["hbm_GBs_per_rank"] = round(model * (r if r else 1.0) / (e["ms"] * 1e-3) / 1e9, 1)
    out["hbm_rate_what"] = ("hbm_GBs_per_rank = staging-model HBM bytes per rank x measured HBM/model ratio "
                            "(profiles/r4/simple_traffic_pmc_r4j.json; 1.0 where unmeasured) / call time")


# bytes over an entry's busiest link, one direction (M = message, n ranks) and
# the probe (push / pull) that prices it: the direct schedules push one block
# to every peer per phase; the ring sends 2 (n-1) blocks to its right
# neighbour over one link; the clique's direct fold pulls block r from every
# peer and pushes the finished block back (both directions at once)
FABRIC_LINK_MODELS = {
    "allreduce_direct": (("push",), lambda n, M: 2 * M // n),
    "transport_allreduce": (("push",), lambda n, M: 2 * M // n),
    "reduce_scatter": (("push",), lambda n, M: M // n),
    "allreduce_ring": (("push",), lambda n, M: 2 * (n - 1) * M // n),
}
FABRIC_CLIQUE_MODELS = {
    "allreduce": (("push",), lambda n, M: 2 * M // n),
    "reduce_scatter": (("push",), lambda n, M: M // n),
    "fold_allreduce": (("pull", "push"), lambda n, M: M // n),
    "fold_reduce_scatter": (("pull",), lambda n, M: M // n),
}


def _fabric_floor(e: dict, kinds, link_bytes: int, rates: dict) -> None:
    if not isinstance(e, dict) or not e.get("ms") or any(k not in rates for k in kinds):
        return
    floor_ms = max(link_bytes / (rates[k] * 1e9) * 1e3 for k in kinds)
    e["fabric_link_bytes"] = link_bytes
    e["fabric_floor_ms"] = round(floor_ms, 4)
    e["fabric_frac"] = round(floor_ms / e["ms"], 3)


def add_fabric_rates(out: dict, allres: list, world: int, msg_bytes: int) -> None:
    """config D against the fabric. Every rank's
    nbxDebugLinkProbe moves the same bytes to (push: the transport's stores)
    or from (pull: its loads) every peer at once; the per-link rate is those
    bytes / the max-over-ranks time. An entry's floor is what its schedule
    moves over its busiest link in one direction / that rate
    (FABRIC_LINK_MODELS), and fabric_frac = floor / the entry's time."""
    n = world
    moved = [r.get("link_bytes_per_peer") for r in allres]
    rates = {}
    for kind in ("push", "pull"):
        ms = [r.get(f"link_{kind}_ms") for r in allres]
        if any(v is None for v in ms + moved) or max(ms) <= 0:
            continue
        rates[kind] = moved[0] / (max(ms) * 1e-3) / 1e9
    if not rates:
        return
    out["fabric"] = {"bytes_per_peer": moved[0],
                     "push_GBs_per_link": round(rates["push"], 2) if "push" in rates else None,
                     "pull_GBs_per_link": round(rates["pull"], 2) if "pull" in rates else None,
                     "push_GBs_per_gpu": round(rates["push"] * (n - 1), 2) if "push" in rates else None,
                     "what": "nbxDebugLinkProbe: every rank moves bytes_per_peer to (push, system-scope stores) or "
                             "from (pull, system-scope loads) every peer's staging at once; per link = bytes / "
                             "max-over-ranks time; entries carry fabric_floor_ms = busiest-link bytes / that rate "
                             "and fabric_frac = floor / time" + (" (ranks share one GPU: the 'links' are its HBM)"
                                                                  if out.get("shared_gpu") else "")}
    out["fabric_rates"] = rates
    for key, (kinds, f) in FABRIC_LINK_MODELS.items():
        _fabric_floor(out.get(key), kinds, f(n, msg_bytes), rates)


def add_clique_fabric(coll: dict, world: int, msg_bytes: int) -> None:
    """The clique's config-D entries against the same per-link rates (the
    clique reaches its peers by direct pointers over the same fabric)."""
    rates = coll.get("fabric_rates")
    cl = coll.get("clique")
    if not rates or not isinstance(cl, dict):
        return
    for key, (kinds, f) in FABRIC_CLIQUE_MODELS.items():
        _fabric_floor(cl.get(key), kinds, f(world, msg_bytes), rates)


def simple_hbm_model(world: int, msg_bytes: int):
    """Per-rank byte model of a config-D Simple AllReduce (both schedules):
    the user-visible bytes, the HBM bytes the staging design moves, and what
    crosses xGMI each way, with the measured HBM / model ratio from the
    committed PMC passes of the same kernels (profiles/r4/simple_traffic_pmc_r4j.json:
    2 ranks on one GPU, one fused dispatch) — carried over, not measured here."""
    n, M = world, msg_bytes
    model = 2 * (M + 2 * (n - 1) * M // n)
    out = {"algorithmic_bytes_per_rank": 2 * M, "staging_model_bytes_per_rank": model,
           "xgmi_bytes_per_rank_each_way": 2 * (n - 1) * M // n,
           "what": "staging model per rank = 2 x (M + 2 (n-1) M / n) HBM bytes (send block into peers' staging; "
                   "fold of own input + n-1 slots into the output and peers' AG staging; gather of n-1 slots)"}
    try:
        with open(os.path.join(ROOT, "profiles", "r4", "simple_traffic_pmc_r4j.json")) as f:
            d = json.load(f)
        out["measured_over_model"] = {k: d[k]["hbm_over_model"] for k in ("direct", "ring")}
        out["measured_provenance"] = ("profiles/r4/simple_traffic_pmc_r4j.json (rocprofv3 FETCH_SIZE / WRITE_SIZE "
                                      "passes, 2 ranks on one GPU); not measured in this run")
    except (OSError, ValueError, KeyError):
        out["measured_over_model"] = None
    return out


def vs_rccl(coll, rccl):
    """libnbxccl time / RCCL time ratios on the same shapes (< 1: libnbxccl faster)."""
    if not coll or not rccl or not rccl.get("ok"):
        return None
    out = {}

    def ratio(ours, theirs):
        return None if ours is None or not theirs else round(ours / theirs, 3)
    ar, rs = coll.get("allreduce_direct"), coll.get("reduce_scatter")
    out["allreduce_1GiB"] = ratio(ar and ar["ms"], rccl.get("allreduce", {}).get("ms"))
    out["reduce_scatter_1GiB"] = ratio(rs and rs["ms"], rccl.get("reduce_scatter", {}).get("ms"))
    out["allreduce_1MiB"] = ratio(coll.get("ll128_allreduce_1MiB_us"), rccl.get("allreduce_1MiB_us"))
    out["allreduce_4KiB"] = ratio(coll.get("ll_allreduce_4KiB_us"), rccl.get("allreduce_4KiB_us"))
    sw, rsw = coll.get("protocol_sweep") or {}, rccl.get("sweep_allreduce_us")
    if sw.get("bytes") and rsw:
        best = []
        for i, b in enumerate(sw["bytes"]):
            cands = [sw[k][i] for k in ("LL", "LL128", "LL128_oneshot", "Simple") if sw.get(k) and i < len(sw[k])]
            j = SWEEP_BYTES.index(b) if b in SWEEP_BYTES else None
            best.append(None if not cands or j is None else round(min(cands) / rsw[j], 3))
        out["sweep_best_protocol"] = best
    cu, rcu = coll.get("allreduce_curve") or {}, rccl.get("curve_allreduce_ms")
    if cu.get("ms") and rcu and len(rcu) == len(cu["ms"]):
        out["allreduce_curve"] = [ratio(a, b) for a, b in zip(cu["ms"], rcu)]
    out["what"] = "libnbxccl time / RCCL time (< 1: libnbxccl faster)"
    return out


def rccl_leg(world: int):
    """RCCL (torch.distributed "nccl" on ROCm) on the same config-D shapes, in
    this process after the collective leg: the vendor library's all-reduce /
    reduce-scatter over the same xGMI links, as the reference point for
    libnbxccl's numbers. Every rank returns the max-over-ranks times."""
    import torch
    import torch.distributed as dist
    if dist.get_backend() != "nccl":
        return None
    out = {"library": "RCCL via torch.distributed (backend nccl)", "ok": True}
    try:
        def timed(fn, iters):
            for _ in range(2):
                fn()
            torch.cuda.synchronize()
            dist.barrier()
            t0 = time.perf_counter()
            for _ in range(iters):
                fn()
            torch.cuda.synchronize()
            return max_over_ranks((time.perf_counter() - t0) / iters, world)
        rank = dist.get_rank()
        x = torch.full((COUNT_D,), float(rank + 1), device="cuda")
        S = COUNT_D * 4
        t = timed(lambda: dist.all_reduce(x), 5)
        out["allreduce"] = {"ms": round(t * 1e3, 4), "algbw_GBs": round(S / t / 1e9, 2),
                            "busbw_GBs": round(S / t / 1e9 * 2 * (world - 1) / world, 2)}
        y = torch.empty(COUNT_D // world, device="cuda")
        x.fill_(float(rank + 1))
        t = timed(lambda: dist.reduce_scatter_tensor(y, x), 5)
        out["reduce_scatter"] = {"ms": round(t * 1e3, 4), "algbw_GBs": round(S / t / 1e9, 2),
                                 "busbw_GBs": round(S / t / 1e9 * (world - 1) / world, 2)}
        want = float(world * (world + 1) // 2)
        if not bool((y == want).all().item()):
            out["ok"] = False
        # xGMI transport alone (reported separately from the reduce):
        # the all-gather of the same 1 GiB moves what the reduce-scatter moves,
        # with no reduction at all
        t = timed(lambda: dist.all_gather_into_tensor(x, y), 5)
        out["allgather_transport"] = {"ms": round(t * 1e3, 4), "algbw_GBs": round(S / t / 1e9, 2),
                                      "busbw_GBs": round(S / t / 1e9 * (world - 1) / world, 2)}
        for name, cnt in (("allreduce_1MiB_us", 256 << 10), ("allreduce_4KiB_us", 1024)):
            z = torch.ones(cnt, device="cuda")
            out[name] = round(timed(lambda: dist.all_reduce(z), 100) * 1e6, 2)
        curve = []
        for b in CURVE_BYTES:
            z = x[:b // 4]
            curve.append(round(timed(lambda: dist.all_reduce(z), 5) * 1e3, 4))
        out["curve_bytes"] = list(CURVE_BYTES)
        out["curve_allreduce_ms"] = curve
        sweep = []
        for b in SWEEP_BYTES:
            z = torch.ones(b // 4, device="cuda")
            sweep.append(round(timed(lambda: dist.all_reduce(z), 50 if b <= (1 << 20) else 20) * 1e6, 2))
        out["sweep_bytes"] = SWEEP_BYTES
        out["sweep_allreduce_us"] = sweep
        del x, y
        torch.cuda.empty_cache()
    except Exception as e:   # reported, never fatal to the bench line
        out = {"ok": False, "errors": [f"{type(e).__name__}: {e}"]}
    return out


COUNT_D = 256 << 20   # config D: fp32 elements per rank (1 GiB)
SWEEP_BYTES = [4 << 10, 32 << 10, 256 << 10, 1 << 20, 4 << 20, 16 << 20]   # = collective_leg.SWEEP_BYTES
CURVE_BYTES = (64 << 20, 256 << 20)   # = collective_leg.CURVE_BYTES: AllReduce between the sweep and config D


def parse_args(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-seconds", type=float, default=1.5)
    ap.add_argument("--check", action="store_true", help="verify step output against the oracle (sampled)")
    return ap.parse_args(argv)


def headline(args, world: int, rank: int, local: int) -> dict:
    """The timed region (config B on this rank's GPU), the roofline fields,
    the same-process stream ceilings and, at N = 1, the host end-to-end leg.
    Returns the result dict (collective / cpu_baseline still None); every
    device buffer of this function is freed when it returns."""
    import torch
    nbx = _load_package()
    nbx.load_library()
    dev = torch.device("cuda", local)

    # inputs resident in HBM before timing: seeded uniform[-1,1) per rank
    g = torch.Generator(device=dev).manual_seed(1234 + 7919 * rank)
    srcs = [torch.rand(COUNT, device=dev, generator=g).mul_(2).sub_(1) for _ in range(N_SRCS)]
    out = torch.empty(COUNT, device=dev)
    stream = torch.cuda.current_stream()
    sh = stream.cuda_stream
    op = nbx.host_to_dev_redop(nbx.ncclRedOp.ncclSum, nbx.ncclDataType.ncclFloat32, 1)
    dptr = [out.data_ptr()]
    sptr = [t.data_ptr() for t in srcs]
    f32 = int(nbx.ncclDataType.ncclFloat32)

    # one step = one nbxReduceMulti launch through the C ABI; the pointer arrays
    # are built once so the host enqueue (~µs) never leaves the GPU idle
    import ctypes
    lib = nbx.load_library()
    d_arr = (ctypes.c_void_p * 1)(*dptr)
    s_arr = (ctypes.c_void_p * N_SRCS)(*sptr)
    sh_c = ctypes.c_void_p(sh)

    def step():
        rc = lib.nbxReduceMulti(d_arr, 1, s_arr, N_SRCS, COUNT, f32, op, 0, 0, sh_c)
        if rc != 0:
            raise RuntimeError(f"nbxReduceMulti failed: {rc}")

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    _barrier(world)
    torch.cuda.synchronize()

    # HIP events on the launch stream bracket the K back-to-back launches (an
    # event between launches costs ~1.5 %: scripts/probe_layout.py)
    evs = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
    t0 = time.perf_counter()
    evs[0].record(stream)
    for i in range(args.steps):
        step()
    evs[1].record(stream)
    torch.cuda.synchronize()
    _barrier(world)
    torch.cuda.synchronize()
    wall = time.perf_counter() - t0
    wall = max_over_ranks(wall, world)
    ms_per_step = wall * 1e3 / args.steps
    kern_avg_ms = evs[0].elapsed_time(evs[1]) / args.steps
    value = world * ALG_BYTES / (wall / args.steps) / 2**30

    if args.check:
        idx = torch.randint(0, COUNT, (1 << 16,), device=dev)
        ref = srcs[0][idx].clone()
        for s in srcs[1:]:
            ref = ref + s[idx]
        assert torch.equal(out[idx], ref), "bench output differs from the left-fold reference"

    achieved = ALG_BYTES / (kern_avg_ms * 1e-3) / 1e9
    # median and best per launch too — a separate pass after the
    # timed region, one event pair per launch (the timed region brackets all K
    # launches with one pair: an event between launches costs ~1.5 %)
    per = []
    for _ in range(max(args.steps, 5)):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(stream)
        step()
        e1.record(stream)
        per.append((e0, e1))
    torch.cuda.synchronize()
    per_ms = sorted(a.elapsed_time(b) for a, b in per)
    traffic, traffic_src = _pmc_traffic()
    ceil = None
    if os.environ.get("NBX_BENCH_CEILING", "1") != "0":
        ceil = stream_ceilings(torch, nbx, srcs, out, stream)
    result = {
        "metric": METRIC,
        "value": round(value, 3),
        "unit": "GiB/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(ms_per_step, 5),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "f32",
        "data": "synthetic (seeded uniform[-1,1) per rank, resident in HBM)",
        "config": {"workload": "config B: 8-input fp32 ncclSum reduce (nbxReduceMulti), 256 MiB per input, "
                               "device-resident; N ranks = N independent shards",
                   "n_srcs": N_SRCS, "count_per_input": COUNT, "bytes_per_step_per_gpu": ALG_BYTES,
                   "parallelism": f"shard{world}"},
        "pct_hbm_peak": round(100.0 * (ALG_BYTES / (wall / args.steps)) / (HBM_PEAK_GBS * 1e9), 2),
        "roofline": {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": round(achieved / HBM_PEAK_GBS, 4), "traffic": traffic,
                     "traffic_provenance": traffic_src,
                     "kernel": "kReducePacks<FnSumF<TyF32>, NSRC=8, U=4>",
                     "tile_schedule": "static" if os.environ.get("NBX_DYNAMIC_TILES", "1") == "0"
                     else "dynamic (per-stream tile counter)",
                     "kernel_avg_ms": round(kern_avg_ms, 5),
                     "kernel_ms_median": round(per_ms[len(per_ms) // 2], 5),
                     "kernel_ms_best": round(per_ms[0], 5),
                     "per_launch_what": f"{len(per_ms)} launches after the timed region, one event pair each",
                     "alg_bytes_per_launch": ALG_BYTES},
        "cpu_baseline": None,
        "collective": None,
        "build": _build_stamp(nbx),
    }
    if ceil:
        rf = result["roofline"]
        rf["ceiling_read"], rf["ceiling_write"], rf["ceiling_copy"] = ceil["read_GBs"], ceil["write_GBs"], ceil["copy_GBs"]
        rf["ceiling_mixed"] = ceil["mixed_GBs"]
        rf["frac_of_ceiling"] = round(achieved / ceil["mixed_GBs"], 4)
        rf["frac_of_read_ceiling"] = round(achieved / max(ceil["read_GBs"], ceil["copy_GBs"]), 4)
        rf["ceiling_what"] = (ceil["what"] + "; frac_of_ceiling = achieved / mixed (the stream the fold faces), "
                              "frac_of_read_ceiling = achieved / max(read, copy)")
    if world > 1:
        # every GPU's own kernel rate (the weak-scaling value hides a straggler)
        import torch.distributed as dist
        mine = {"rank": rank, "device": local, "kernel_avg_ms": round(kern_avg_ms, 5),
                "kernel_GBs": round(achieved, 1)}
        every = [None] * world
        dist.all_gather_object(every, mine)
        result["per_rank"] = every
    if world == 1 and os.environ.get("NBX_BENCH_E2E", "1") != "0" and not args.no_cpu_baseline:
        result["host_e2e"] = host_e2e_leg(torch, nbx, srcs, out, stream, op)
    del srcs, out
    torch.cuda.empty_cache()
    return result


def run_legs(result: dict, world: int, rank: int, local: int, child, clique_child, emitter: Emitter,
             budget: LegBudget) -> dict | None:
    """The N > 1 legs inside one wall budget (module docstring); rank 0
    returns the collective summary, the other ranks None."""
    emitter.leg = "the collective leg"
    # the multi-process leg may use what the clique and RCCL legs do not need
    coll = collective_leg(child, world, rank, budget=budget, reserve=2 * LEG_MIN_S)
    emitter.coll = coll
    if os.environ.get("NBX_BENCH_CLIQUE", "1") != "0":
        emitter.leg = "the clique leg"
        cl = clique_leg(clique_child, world, rank, local, budget=budget)
        if coll is not None:
            coll["clique"] = cl
            add_clique_fabric(coll, world, COUNT_D * 4)
    if os.environ.get("NBX_BENCH_RCCL", "1") != "0":
        emitter.leg = "the RCCL leg"
        left = budget.agreed_left(world)
        rccl = rccl_leg(world) if left >= LEG_MIN_S else skipped_leg(left, "the RCCL leg")
        if coll is not None:
            coll["rccl"] = rccl
            coll["vs_rccl"] = vs_rccl(coll, rccl)
    emitter.leg = None
    if coll is not None:
        coll["leg_budget"] = {"budget_s": budget.total, "used_s": round(budget.total - budget.left(), 1)}
        coll.pop("fabric_rates", None)
    return coll


def main(argv=None):
    args = parse_args(argv)
    env_world = int(os.environ.get("WORLD_SIZE", "1"))
    child = _spawn_collective_leg(env_world)
    clique_child = _spawn_clique_leg(env_world, int(os.environ.get("RANK", "0")))
    import torch
    world, rank, local = _dist_init()
    if args.gpus != world and world > 1:
        print(f"warning: --gpus {args.gpus} but WORLD_SIZE {world}", file=sys.stderr)
    emitter = Emitter(rank)
    result = headline(args, world, rank, local)
    emitter.result = result
    if child is not None:
        # the headline first: whatever the legs do, the value is on stdout
        emitter.preliminary(result)
        budget = LegBudget()
        wd = Watchdog(budget.total + WATCHDOG_GRACE_S, emitter, [child, clique_child])
        result["collective"] = run_legs(result, world, rank, local, child, clique_child, emitter, budget)
        wd.cancel()
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        result["cpu_baseline"] = cpu_baseline(args.cpu_seconds)
    emitter.final(result)
    if world > 1:
        import torch.distributed as dist
        dist.destroy_process_group()
    return EXIT_LEG_CUT_OFF if rank == 0 and legs_cut_off(result.get("collective")) else 0


if __name__ == "__main__":
    sys.exit(main())
