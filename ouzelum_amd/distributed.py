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


def shard(num_envs_local, rank, world):
    """(env_id_offset, num_envs_total) for this rank."""
    return rank * num_envs_local, world * num_envs_local


def allreduce_returns(stats):
    """All-reduce a [sum, count] float64 tensor in place; returns the global mean return."""
    if dist.is_available() and dist.is_initialized() and dist.get_world_size() > 1:
        dist.all_reduce(stats, op=dist.ReduceOp.SUM)
    s, c = stats.tolist()
    return s / c if c > 0 else float("nan")


class GraphCollectives:
    """The row-range all-reduces of a ``ReturnAllReduce`` slot block, captured once as hipGraphs and launched
    through raw HIP calls on a collective stream of their own.

    An eager ``dist.all_reduce(async_op=True)`` costs 14-22 us of host time (ProcessGroupNCCL's work object,
    events and stream bookkeeping around the RCCL call; measured on a one-rank group, where RCCL itself does
    nothing for an in-place reduction: ``profiles/r03/allreduce_graph.jsonl``).  Every flush of a block is a
    fixed row range [lo, hi) of a fixed buffer, so all of them can be captured at construction (depth x
    batch (batch + 1) / 2 graphs, ~0.05 ms of capture each); a flush then costs four HIP calls -- record
    an event on the caller's stream, make the collective stream wait for it, ``hipGraphLaunch``, record the
    graph's completion event -- and a wait one ``hipStreamWaitEvent``.  RCCL supports stream capture;
    every rank replays the same graphs in the same order, exactly as it would call the collectives.
    """

    LIB = os.path.join(os.path.dirname(torch.__file__), "lib", "libamdhip64.so")

    def __init__(self, slots):
        import ctypes
        self._ct = ctypes
        self.hip = ctypes.CDLL(self.LIB)
        dev = slots.device
        self.cs = torch.cuda.Stream(device=dev)
        self._cs = ctypes.c_void_p(self.cs.cuda_stream)
        self._dev = dev
        depth, batch = slots.shape[0], slots.shape[1]
        cur = torch.cuda.current_stream(dev)
        self.cs.wait_stream(cur)
        with torch.cuda.stream(self.cs):
            dist.all_reduce(slots[0, :1], op=dist.ReduceOp.SUM)   # communicator set up outside the capture
            self.graphs = {}
            for d in range(depth):
                for lo in range(batch):
                    for hi in range(lo + 1, batch + 1):
                        g = torch.cuda.CUDAGraph()
                        g.capture_begin(capture_error_mode="thread_local")
                        try:
                            dist.all_reduce(slots[d, lo:hi], op=dist.ReduceOp.SUM)
                        finally:
                            g.capture_end()
                        self.graphs[(d, lo, hi)] = (g, ctypes.c_void_p(g.raw_cuda_graph_exec()), self._event())
        cur.wait_stream(self.cs)
        self._ev_in = self._event()

    def _event(self):
        e = self._ct.c_void_p()
        if self.hip.hipEventCreateWithFlags(self._ct.byref(e), 2) != 0:   # hipEventDisableTiming
            raise RuntimeError("hipEventCreateWithFlags failed")
        return e

    def _check(self, err, what):
        if err != 0:
            raise RuntimeError(f"{what} failed (hipError {err})")

    def launch(self, d, lo, hi):
        """Reduce rows [lo, hi) of block d after the work queued so far on the caller's stream; returns the
        completion event."""
        from . import _lib
        _, ex, done = self.graphs[(d, lo, hi)]
        s = self._ct.c_void_p(_lib.stream_ptr(self._dev))
        self._check(self.hip.hipEventRecord(self._ev_in, s), "hipEventRecord")
        self._check(self.hip.hipStreamWaitEvent(self._cs, self._ev_in, 0), "hipStreamWaitEvent")
        self._check(self.hip.hipGraphLaunch(ex, self._cs), "hipGraphLaunch")
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
        for _, _, e in getattr(self, "graphs", {}).values():
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
    eager call of ``dist.all_reduce`` costs 14-22 us of host time (RCCL, ``profiles/r01/allreduce_host.txt``,
    ``profiles/r03/allreduce_graph.jsonl``), as much as five 4096-env steps, so ``batch`` rollouts
    share it; the per-rollout global statistics are unchanged.  ``collective="graph"`` (the default on
    the "nccl" backend, i.e. RCCL) replays pre-captured hipGraphs of the same collectives instead
    (``GraphCollectives``, a few us of host time per flush); it is checked against the eager form at
    construction on every rank and falls back to eager, on all ranks together, if the check fails.
    ``OUZ_COLLECTIVE=eager`` forces the eager form.  A block is only reused after its
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
        self.graphs = None
        if collective is None:
            collective = os.environ.get("OUZ_COLLECTIVE", "graph")
        if collective not in ("graph", "eager"):
            raise ValueError(f"collective must be 'graph' or 'eager', not {collective!r}")
        if (self.active and collective == "graph" and self.slots.is_cuda
                and dist.get_backend() == dist.Backend.NCCL):
            self.graphs = self._graph_collectives()
        self.collective = "graph" if self.graphs is not None else "eager"

    def _graph_collectives(self):
        """Capture the block collectives and check them once against the known sums; every rank takes the
        same decision (an eager all-reduce of the verdicts)."""
        rank, world = dist.get_rank(), dist.get_world_size()

        def agree(ok):   # eager all-reduce of the ranks' verdicts: every rank takes the same branch
            v = torch.tensor([1.0 if ok else 0.0], dtype=torch.float64, device=self.slots.device)
            dist.all_reduce(v, op=dist.ReduceOp.MIN)
            return v.item() == 1.0

        try:
            g = GraphCollectives(self.slots)
        except Exception:   # noqa: BLE001 -- a capture failure means: use the eager collectives
            g = None
        if not agree(g is not None):   # captured graphs run no collective: the ranks are still in step here
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
            if self.graphs is not None:
                self.graphs.wait(w)
            else:
                w.wait()
        self.works[d] = []

    def _flush(self, d, hi):
        if self.active and self.lo[d] < hi:
            if self.graphs is not None:
                self.works[d].append(self.graphs.launch(d, self.lo[d], hi))
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
            self._flush(d, self.filled[d])
            self._wait(d)

    def result(self, r):
        d, row = self._where(r)
        self._flush(d, row + 1)
        self._wait(d)
        return self.slots[d, row]
