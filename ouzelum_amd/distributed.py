"""One process per GPU: env sharding and the single RCCL collective of the path.

Envs are independent, so the step itself never communicates.
Rank r simulates global env ids [r*N_local, (r+1)*N_local); every random draw
and the PV-filter trigger index are keyed on the global id, so trajectories do
not depend on the GPU count.  The only exchange is one all-reduce of
[sum of finished-episode returns, episode count] per rollout — the analogue of
rl_games' Horovod stat averaging (learning/common_agent.py:137,218-240) —
over torch.distributed's "nccl" backend, which is RCCL over xGMI on MI355X.
"""
import os

import torch
import torch.distributed as dist


def init_from_env(backend=None):
    """Initialise torch.distributed from torchrun's env vars; returns (rank, world, local_rank)."""
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1 and not dist.is_initialized():
        if backend is None:
            # OUZ_DIST_BACKEND=gloo: rehearse the N > 1 path with several ranks on one GPU (RCCL wants
            # one GPU per rank); the product path is "nccl" = RCCL over xGMI
            backend = os.environ.get("OUZ_DIST_BACKEND") or ("nccl" if torch.cuda.is_available() else "gloo")
        if backend == "nccl":
            torch.cuda.set_device(local)
            dist.init_process_group(backend, device_id=torch.device("cuda", local))
        else:
            dist.init_process_group(backend)
    return rank, world, local


def loaded_library(stem):
    """Path of a shared library this process has ALREADY mapped whose file name starts with ``stem`` (e.g.
    "libamdhip64.so", "librccl.so"), from /proc/self/maps, or None.  The direct collectives and the bench's raw
    events call into the runtime torch itself loaded: opening another copy by path (torch/lib against
    /opt/rocm/lib) would give a second HIP / RCCL runtime, whose calls on torch's streams and communicator
    crash instead of failing."""
    try:
        with open("/proc/self/maps") as fh:
            for line in fh:
                parts = line.split()
                if len(parts) >= 6 and os.path.basename(parts[5]).startswith(stem):
                    return parts[5]
    except OSError:  # pragma: no cover - not Linux
        return None
    return None


def _comm_ptr(dev):
    """The ncclComm_t of the default process group's RCCL backend on ``dev`` (0 if unavailable).  This goes
    through torch's private ProcessGroup API (``_get_backend(dev)._comm_ptr()``, present in torch 2.4-2.10);
    any other torch raises AttributeError / RuntimeError here and the callers fall back."""
    grp = dist.distributed_c10d._get_default_group()
    be = grp._get_backend(dev)
    fn = getattr(be, "_comm_ptr", None)
    if fn is None:
        raise AttributeError(f"torch {torch.__version__}: ProcessGroupNCCL has no _comm_ptr()")
    return int(fn())


def rccl_comm_count(dev):
    """Ranks of the RCCL communicator the process group runs its collectives on (``ncclCommCount``), or None
    when the backend is not RCCL or the communicator cannot be reached."""
    import ctypes
    if not (dist.is_available() and dist.is_initialized()) or dist.get_backend() != dist.Backend.NCCL:
        return None
    try:
        comm = _comm_ptr(dev)
        path = loaded_library("librccl.so")
        if not comm or not path:
            return None
        rccl = ctypes.CDLL(path, mode=getattr(os, "RTLD_NOLOAD", 4) | ctypes.RTLD_GLOBAL)
        cnt = ctypes.c_int(0)
        rccl.ncclCommCount.argtypes = [ctypes.c_void_p, ctypes.POINTER(ctypes.c_int)]
        if rccl.ncclCommCount(ctypes.c_void_p(comm), ctypes.byref(cnt)) != 0:
            return None
        return int(cnt.value)
    except Exception:  # noqa: BLE001 -- a report field, never a reason to fail the run
        return None


def shard(num_envs_local, rank, world):
    """(env_id_offset, num_envs_total) for this rank."""
    return rank * num_envs_local, world * num_envs_local


def allreduce_returns(stats):
    """All-reduce a [sum, count] float64 tensor in place; returns the global mean return."""
    if dist.is_available() and dist.is_initialized() and dist.get_world_size() > 1:
        dist.all_reduce(stats, op=dist.ReduceOp.SUM)
    s, c = stats.tolist()
    return s / c if c > 0 else float("nan")


class DirectCollectives:
    """The flushes of a ``ReturnAllReduce`` slot block as direct RCCL calls on the communicator the process
    group already holds, on a collective stream of their own.

    Host cost of one flush (``scripts/exp/allreduce_graph.py``, ``profiles/r03/allreduce_host.jsonl``, medians of
    per-call times on two boxes): ``dist.all_reduce(async_op=True)`` 13-20 us (ProcessGroupNCCL's work object,
    events and stream bookkeeping); the collective captured in a hipGraph and replayed behind an event pair
    12-14 us (``hipGraphLaunch`` of a one-kernel graph alone is 7-9 us on this ROCm); this form behind the
    event pair 7-12 us (each ``hipEventRecord`` 1.7-2.3 us); this form in the caller's stream 1.2 us (one
    rank: RCCL enqueues nothing) to 4.5 us (with one device operation enqueued, the stand-in for the RCCL
    kernel of a multi-rank call).  The asynchronous flush of a full block (``submit``) goes behind the event
    pair on the collective stream, so the next rollouts step while it runs; a flush the caller waits for
    next (``finish``, ``result``) goes in the caller's stream.  Every rank makes the same calls in the same
    order, exactly as it would call ``dist.all_reduce``; RCCL runs a communicator's operations in that order
    whatever stream they are on.
    """

    NCCL_FLOAT64, NCCL_SUM = 8, 0   # ncclDataType_t / ncclRedOp_t values of nccl.h (RCCL keeps NCCL's enums)

    def __init__(self, slots):
        import ctypes
        self._ct = ctypes
        hip_path, rccl_path = loaded_library("libamdhip64.so"), loaded_library("librccl.so")
        if not hip_path or not rccl_path:
            raise RuntimeError("the HIP / RCCL runtimes torch loaded are not mapped in this process")
        noload = getattr(os, "RTLD_NOLOAD", 4)
        self.hip = ctypes.CDLL(hip_path, mode=noload | ctypes.RTLD_GLOBAL)
        self.rccl = ctypes.CDLL(rccl_path, mode=noload | ctypes.RTLD_GLOBAL)
        self.rccl.ncclAllReduce.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int,
                                            ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p]
        self.rccl.ncclAllReduce.restype = ctypes.c_int
        dev = slots.device
        self._dev = dev
        self.cs = torch.cuda.Stream(device=dev)
        self._cs = ctypes.c_void_p(self.cs.cuda_stream)
        comm = _comm_ptr(dev)
        if not comm:
            raise RuntimeError("the process group has no RCCL communicator")
        self._comm = ctypes.c_void_p(comm)
        self._base = slots.data_ptr()
        self._width = slots.shape[2]
        self._batch = slots.shape[1]
        self._ev_in = self._event()
        self._done = [[self._event() for _ in range(slots.shape[1])] for _ in range(slots.shape[0])]

    def _event(self):
        e = self._ct.c_void_p()
        if self.hip.hipEventCreateWithFlags(self._ct.byref(e), 2) != 0:   # hipEventDisableTiming
            raise RuntimeError("hipEventCreateWithFlags failed")
        return e

    @staticmethod
    def _check(err, what):
        if err != 0:
            raise RuntimeError(f"{what} failed (error {err})")

    def launch(self, d, lo, hi, in_stream=False):
        """Sum rows [lo, hi) of block d over the ranks, after the work queued so far on the caller's stream;
        returns the completion event.  in_stream: on the caller's stream itself (for a caller about to wait
        for the result anyway: one RCCL call, no event pair); returns None."""
        from . import _lib
        done = self._done[d][lo]
        s = self._ct.c_void_p(_lib.stream_ptr(self._dev))
        p = self._ct.c_void_p(self._base + ((d * self._batch + lo) * self._width) * 8)
        if in_stream:
            self._check(self.rccl.ncclAllReduce(p, p, (hi - lo) * self._width, self.NCCL_FLOAT64, self.NCCL_SUM,
                                                self._comm, s), "ncclAllReduce")
            return None
        self._check(self.hip.hipEventRecord(self._ev_in, s), "hipEventRecord")
        self._check(self.hip.hipStreamWaitEvent(self._cs, self._ev_in, 0), "hipStreamWaitEvent")
        self._check(self.rccl.ncclAllReduce(p, p, (hi - lo) * self._width, self.NCCL_FLOAT64, self.NCCL_SUM,
                                            self._comm, self._cs), "ncclAllReduce")
        self._check(self.hip.hipEventRecord(done, self._cs), "hipEventRecord")
        return done

    def wait(self, done):
        """Order the caller's stream after a launch's completion event."""
        from . import _lib
        s = self._ct.c_void_p(_lib.stream_ptr(self._dev))
        self._check(self.hip.hipStreamWaitEvent(s, done, 0), "hipStreamWaitEvent")

    def __del__(self):
        hip = getattr(self, "hip", None)
        if hip is None:
            return
        for row in getattr(self, "_done", []):
            for e in row:
                hip.hipEventDestroy(e)
        if getattr(self, "_ev_in", None):
            hip.hipEventDestroy(self._ev_in)


class ReturnAllReduce:
    """The per-rollout return all-reduce taken off the stepping critical path.

    ``allreduce_returns`` is blocking in stream order: the next rollout's step kernels wait for
    the collective (an 8-byte RCCL all-reduce over xGMI is latency-bound, ~10-30 us on 8 GPUs,
    i.e. several 4096-env steps).  Nothing the env does depends on the reduced value, so this
    helper keeps ``depth`` blocks of ``batch`` stat rows: rollout r's stats go to row r % batch of
    block (r // batch) % depth, and a block is all-reduced asynchronously, in ONE collective, once
    its last row is submitted, on the collective's own stream while the next rollouts step.  One
    eager call of ``dist.all_reduce`` costs 13-22 us of host time (RCCL, ``profiles/r01/allreduce_host.txt``,
    ``profiles/r03/allreduce_host.jsonl``), as much as five 4096-env steps, so ``batch`` rollouts
    share it; the per-rollout global statistics are unchanged.  ``collective="direct"`` (opt-in on the
    "nccl" backend, i.e. RCCL, with ``OUZ_COLLECTIVE=direct``) issues the same collectives as direct RCCL calls
    on the process group's communicator instead (``DirectCollectives``, about half the host time per flush); it
    is checked at construction on every rank and falls back to eager, on all ranks together, if the check
    fails.  The default is ``eager`` (``dist.all_reduce``): the direct form has only run on a one-rank RCCL
    communicator, and until a run on two or more GPUs validates it, the product path uses torch's own.  A block is only reused after its
    collectives have completed (``wait`` orders the current stream after them).  ``result(r)``
    returns the global [sum, count, ...] of rollout r, flushing the rows not yet reduced first;
    every rank must make the same calls in the same order (they are collectives).
    """

    def __init__(self, device, depth=2, width=3, batch=1, collective=None):
        if depth < 1 or batch < 1:
            raise ValueError("depth and batch must be >= 1")
        self.slots = torch.zeros((depth, batch, width), dtype=torch.float64, device=device)
        self.depth, self.batch = depth, batch
        self.works = [[] for _ in range(depth)]
        self.lo = [0] * depth       # first row of the block not yet in a submitted collective
        self.filled = [0] * depth   # rows of the block submitted by the caller
        self.active = dist.is_available() and dist.is_initialized() and dist.get_world_size() > 1
        self._base = None
        self._row_bytes = width * self.slots.element_size()
        self.direct = None
        if collective is None:
            collective = os.environ.get("OUZ_COLLECTIVE", "eager")
        if collective not in ("direct", "eager"):
            raise ValueError(f"collective must be 'direct' or 'eager', not {collective!r}")
        if (self.active and collective == "direct" and self.slots.is_cuda
                and dist.get_backend() == dist.Backend.NCCL):
            self.direct = self._direct_collectives()
        self.collective = "direct" if self.direct is not None else "eager"

    def _direct_collectives(self):
        """Set up the direct collectives and check them once against the known sums; every rank takes the
        same decision (an eager all-reduce of the verdicts)."""
        rank, world = dist.get_rank(), dist.get_world_size()

        def agree(ok):   # eager all-reduce of the ranks' verdicts: every rank takes the same branch
            v = torch.tensor([1.0 if ok else 0.0], dtype=torch.float64, device=self.slots.device)
            dist.all_reduce(v, op=dist.ReduceOp.MIN)
            return v.item() == 1.0

        dist.all_reduce(self.slots[0, :1], op=dist.ReduceOp.SUM)   # every rank: the communicator exists
        torch.cuda.synchronize(self.slots.device)
        try:
            g = DirectCollectives(self.slots)
        except Exception:   # noqa: BLE001 -- a setup failure means: use the eager collectives
            g = None
        if not agree(g is not None):   # the setup runs no collective: the ranks are still in step here
            return None
        ok = True
        try:
            want = world * (world + 1) / 2
            for lo, hi in ((0, self.batch), (self.batch // 2, self.batch)):
                for d in range(self.depth):
                    self.slots[d].fill_(rank + 1.0)
                    g.wait(g.launch(d, lo, hi))
                    got = self.slots[d].cpu()
                    expect = torch.full_like(got, rank + 1.0)
                    expect[lo:hi] = want
                    ok = ok and torch.equal(got, expect)
        except Exception:   # noqa: BLE001
            ok = False
        torch.cuda.synchronize(self.slots.device)
        ok = agree(ok)
        self.slots.zero_()
        torch.cuda.synchronize(self.slots.device)
        return g if ok else None

    def _where(self, r):
        return (r // self.batch) % self.depth, r % self.batch

    def _wait(self, d):
        for w in self.works[d]:
            if self.direct is not None:
                self.direct.wait(w)
            else:
                w.wait()
        self.works[d] = []

    def _flush(self, d, hi, now=False):
        """now: the caller waits for these rows next (finish / result), so the direct form reduces them in its
        stream (one RCCL call, ~1-5 us of host time) instead of on the collective stream behind an event pair."""
        if self.active and self.lo[d] < hi:
            if self.direct is not None:
                if now:
                    self._wait(d)   # the block's earlier rows first: the calls stay in the same order everywhere
                    self.direct.launch(d, self.lo[d], hi, in_stream=True)
                else:
                    self.works[d].append(self.direct.launch(d, self.lo[d], hi))
            else:
                self.works[d].append(dist.all_reduce(self.slots[d, self.lo[d]:hi], op=dist.ReduceOp.SUM,
                                                     async_op=True))
        self.lo[d] = max(self.lo[d], hi)

    def slot(self, r):
        """The output row for rollout r (a block's first row waits for that block's previous collectives)."""
        d, row = self._where(r)
        if row == 0:
            self._wait(d)
            self.lo[d] = self.filled[d] = 0
        return self.slots[d, row]

    def slot_ptr(self, r):
        """Device address of ``slot(r)`` (the same waiting), for C entry points that take a double*."""
        if not self.active:   # one rank: no collectives to wait for (the call sits before a timed launch)
            if self._base is None:
                self._base = self.slots.data_ptr()
            return self._base + ((r // self.batch) % self.depth * self.batch + r % self.batch) * self._row_bytes
        d, row = self._where(r)
        if row == 0:
            self._wait(d)
            self.lo[d] = self.filled[d] = 0
        if self._base is None:
            self._base = self.slots.data_ptr()
        return self._base + (d * self.batch + row) * self.slots.shape[2] * 8

    def submit(self, r):
        if not self.active:
            return
        d, row = self._where(r)
        self.filled[d] = max(self.filled[d], row + 1)
        if row == self.batch - 1:
            self._flush(d, self.batch)

    def finish(self):
        if not self.active:
            return
        for d in range(self.depth):
            self._flush(d, self.filled[d], now=True)
            self._wait(d)

    def result(self, r):
        d, row = self._where(r)
        self._flush(d, row + 1, now=True)
        self._wait(d)
        return self.slots[d, row]
