"""Multi-file, multi-GPU batch driver (BASELINE.json configs 4 and 5).

The reference processes the files of a batch strictly one after another
(main.cp:132-147), each through process_file (ProcessFile.cp:27-120).  Here
one process per GPU takes a share of the batch:

  * num_files >= world: whole files, round-robin -- "one file per GPU" when
    num_files == world.  The filtering needs no collective: files are
    independent.  With --normalize (config 5) the ranks still MAX all-reduce
    the [num_files] peak vector (each rank fills its own files' slots, the
    rest stay 0, so every file keeps its own peak): the step ends with every
    rank holding the batch's per-file peaks, the RCCL peak exchange
    BASELINE.json's config 5 names, without changing any file's result.
  * num_files < world: each file is split by sample range over a group of
    ranks (each rank reads its range +- half the kernel, no halo exchange).
    The per-file peak is then the max over the group: that is the one real
    exchange step, a MAX all-reduce of the [num_files] peak vector (each
    rank writes its own slots).  Over RCCL/xGMI it is a few dozen bytes.

Normalize semantics follow the reference: per FILE (ProcessFile.cp:92-101,
peak over the file's channels, rescale iff peak > 1 or --normalize).
peak_scope="global" is the north-star config-5 variant (one peak over the
whole batch, RCCL MAX all-reduce, every file rescaled by it) -- a deviation
from the reference, offered only behind that explicit flag.

Compute is pluggable (`Backend`): DeviceBackend runs the gfx950 kernels via
the C ABI on torch-allocated HBM; tests plug a CPU backend built on the
oracle to check the sharding and exchange logic with gloo.
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import Callable, Dict, List, Optional, Sequence


@dataclass(frozen=True)
class Shard:
    file: int
    start: int  # output range [start, end) of every channel of the file
    end: int


def plan_shards(nframes: Sequence[int], world: int) -> List[List[Shard]]:
    """Shards per rank.  Files are whole when num_files >= world, otherwise
    split into contiguous near-equal ranges over ranks (ProcessFile.cp:64-69
    partition rule: chunk = n / parts, the last part takes the remainder)."""
    nf = len(nframes)
    out: List[List[Shard]] = [[] for _ in range(world)]
    if nf == 0:
        return out
    if nf >= world:
        for f, n in enumerate(nframes):
            out[f % world].append(Shard(f, 0, int(n)))
        return out
    # nf < world: ranks [first_f, first_{f+1}) serve file f
    base, extra = divmod(world, nf)
    r = 0
    for f, n in enumerate(nframes):
        parts = base + (1 if f < extra else 0)
        chunk = int(n) // parts
        for i in range(parts):
            s = i * chunk
            e = int(n) if i == parts - 1 else s + chunk
            out[r].append(Shard(f, s, e))
            r += 1
    return out


def file_is_split(plan: List[List[Shard]]) -> bool:
    owners: Dict[int, int] = {}
    for rank, shards in enumerate(plan):
        for sh in shards:
            if owners.setdefault(sh.file, rank) != rank:
                return True
    return False


def window(sh: Shard, n: int, half: int):
    """Samples [x_lo, x_hi) a shard's outputs read (FilterCore.h:56-76)."""
    return max(0, sh.start - half), min(n, sh.end + half)


class Backend:
    """Compute interface the driver needs (device or test CPU)."""

    def upload(self, file: int, xw, x_lo: int, x_hi: int):  # -> handle
        raise NotImplementedError

    def alloc_out(self, nch: int, count: int):  # -> handle
        raise NotImplementedError

    def window(self, n: int, start: int, end: int, half: int):
        """Input samples [x_lo, x_hi) to read for outputs [start, end)."""
        return window(Shard(-1, start, end), n, half)

    def filter(self, xw, x_lo, x_hi, n, nch, yw, start, end, peaks, slot: int):
        """outputs [start, end) into yw; max|y| over the shard's channels into peaks[slot]."""
        raise NotImplementedError

    def zero_peaks(self, peaks):
        raise NotImplementedError

    def normalize(self, yw, nch, count, peaks, slot: Optional[int], force: bool):
        """rescale by 1/peak iff peak > 1 or force; slot None = max over all slots."""
        raise NotImplementedError

    def normalize_clear(self, yw, nch, count, peaks, slot: Optional[int], force: bool, clear):
        """normalize, then zero the (separate) peak vector `clear`."""
        self.normalize(yw, nch, count, peaks, slot, force)
        self.zero_peaks(clear)

    def filter_normalize_prev(self, xw, x_lo, x_hi, n, nch, yw, start, end, peaks, slot: int,
                              prev_yw, prev_count: int, prev_peaks, prev_slot: Optional[int], force: bool):
        """filter, plus an earlier shard's per-file normalize (its peak in
        prev_peaks[prev_slot], final already; prev_slot None = max over all
        slots).  A device backend fuses the two into one launch."""
        self.filter(xw, x_lo, x_hi, n, nch, yw, start, end, peaks, slot)
        self.normalize(prev_yw, nch, prev_count, prev_peaks, prev_slot, force)

    def new_peaks(self, nfiles: int):
        raise NotImplementedError

    def set_lane(self, lane: int):
        """issue what follows on pipeline lane `lane` (BatchRunner(lanes > 1))."""

    def join_lanes(self):
        """every lane's later work follows everything issued so far on every lane."""

    def retain(self, handle, lane: int):
        """`handle` is used by work issued on `lane`: keep its memory alive
        until that work is done even if the caller drops it first."""

    def publish(self, lane: int):
        """the caller's current stream waits for everything issued on `lane`."""



class BatchRunner:
    """One rank's share of a batch.  prepare() uploads the rank's sample
    windows (untimed); step() is the timed per-batch compute: filter every
    shard with fused peaks, exchange peaks if needed, normalize.

    lanes > 1 pipelines consecutive steps: step k is issued on lane k mod
    lanes (its own stream, output buffers and peak vectors), so on the device
    a step's first segments run on the CUs the previous step's last round
    leaves idle.  Steps of one lane stay in order; results() is the latest
    step's outputs.

    Where the normalize goes (ProcessFile.cp:91-101, per file):
      * no peak exchange: a file's peak is final when its own filter is done,
        so its normalize rides in the NEXT shard's filter launch of the same
        step (fuse); only the last shard's runs as a pass of its own;
      * with a peak exchange (config 5 over ranks, split files, global scope):
        every normalize must wait for the all-reduce, so each shard's normalize
        rides in the same shard's filter launch of the lane's NEXT step
        (defer).  A step then is filter launches + the all-reduce, with no
        pass of its own; the outputs alternate between two buffer sets per
        lane, and results() / close() run the normalizes still pending
        (flush) before anyone reads the outputs.
    force_exchange runs the all-reduce even where the plan needs none (world
    1: it exercises the collective on the device, RCCL included)."""

    def __init__(self, backend: Backend, rank: int, world: int, nframes: Sequence[int], nch: int,
                 half: int, normalize: bool = False, peak_scope: str = "file",
                 allreduce_max: Optional[Callable] = None, lanes: int = 1,
                 fuse_normalize: bool = True, force_exchange: bool = False):
        if peak_scope not in ("file", "global"):
            raise ValueError("peak_scope must be 'file' or 'global'")
        if lanes < 1:
            raise ValueError("lanes must be >= 1")
        self.b = backend
        self.rank, self.world = rank, world
        self.nframes = [int(n) for n in nframes]
        self.nch, self.half = nch, half
        self.normalize = normalize
        self.scope = peak_scope
        self.plan = plan_shards(self.nframes, world)
        self.shards = self.plan[rank]
        split = file_is_split(self.plan)
        # the collective: where files share ranks (a file's peak is the max
        # over its ranks), for the batch-global variant, and with --normalize
        # (config 5: every rank learns every file's peak; zeros elsewhere keep
        # each file's own peak, ProcessFile.cp:92-101)
        self.exchange = force_exchange or (world > 1 and (split or peak_scope == "global" or normalize))
        if self.exchange and allreduce_max is None:
            raise ValueError("this plan needs a MAX all-reduce of the peak vector")
        self.allreduce_max = allreduce_max
        # Without an exchange, a file's peak is final when its own filter is
        # done: its normalize then rides in the NEXT shard's filter launch
        # (Backend.filter_normalize_prev) and only the last shard's runs as a
        # pass of its own.  With an exchange every normalize waits for it.
        self.fuse = fuse_normalize and not self.exchange and peak_scope == "file"
        # With an exchange, each normalize rides in the lane's next step instead.
        self.defer = fuse_normalize and self.exchange
        # Per lane, peak vectors rotating by step: a step's last normalize
        # launch (or, deferred, a reset after the all-reduce) zeroes the next
        # step's, so no separate reset launch sits in a step.  Deferred, a
        # step's vector is still read by the next step: three in rotation.
        self.lanes = lanes
        self._nvec = 3 if self.defer else 2
        self._nsets = 2 if self.defer else 1  # output buffer sets per lane
        self._peak_bufs = [[backend.new_peaks(len(self.nframes)) for _ in range(self._nvec)]
                           for _ in range(lanes)]
        self._steps = [0] * lanes  # steps issued per lane since prepare()
        self._pending = [None] * lanes  # defer: (outputs, peaks) of the lane's last step, not normalized
        self._lane = 0
        self._last = 0
        self.peaks = self._peak_bufs[0][0]  # the most recent step's per-file peaks
        self.inputs = []
        self.outputs = []
        self._outs = [[[] for _ in range(self._nsets)] for _ in range(lanes)]

    def prepare(self, get_window: Callable):
        """get_window(file, x_lo, x_hi) -> [nch][x_hi - x_lo] float32 samples."""
        self.inputs = []
        self._outs = [[[] for _ in range(self._nsets)] for _ in range(self.lanes)]
        self._pending = [None] * self.lanes
        self.b.join_lanes()  # a re-prepare waits for steps still in flight on any lane
        self.b.set_lane(0)
        for bufs in self._peak_bufs:
            for pk in bufs:
                self.b.zero_peaks(pk)
        for sh in self.shards:
            n = self.nframes[sh.file]
            lo, hi = self.b.window(n, sh.start, sh.end, self.half)
            xw = self.b.upload(sh.file, get_window(sh.file, lo, hi), lo, hi)
            self.inputs.append((xw, lo, hi))
            for lane, sets in enumerate(self._outs):
                self.b.retain(xw, lane)
                for outs in sets:
                    outs.append(self.b.alloc_out(self.nch, sh.end - sh.start))
                    self.b.retain(outs[-1], lane)
        for lane, bufs in enumerate(self._peak_bufs):
            for pk in bufs:
                self.b.retain(pk, lane)
        self.outputs = self._outs[0][0]
        self.b.join_lanes()
        self._steps = [0] * self.lanes
        self._lane = 0
        self._last = 0

    def output_buffer(self, lane: int, index: int, which: int = 0):
        """Output handle of shard `index` in buffer set `which` of `lane`."""
        return self._outs[lane][which][index]

    def output_buffer_set(self, lane: int, which: int = 0):
        """Every shard's output handle in buffer set `which` of `lane`."""
        return list(self._outs[lane][which])

    def _slot(self, sh: Shard) -> Optional[int]:
        return None if self.scope == "global" else sh.file

    def step(self):
        lane = self._lane
        self.b.set_lane(lane)
        k = self._steps[lane]
        outputs = self._outs[lane][k % self._nsets]
        peaks = self._peak_bufs[lane][k % self._nvec]        # zero (prepare, or the lane's previous step)
        nxt = self._peak_bufs[lane][(k + 1) % self._nvec]    # the lane's next step's: zeroed by this step
        pend = self._pending[lane]
        prev = None
        for i, (sh, (xw, lo, hi), yw) in enumerate(zip(self.shards, self.inputs, outputs)):
            n = self.nframes[sh.file]
            if pend is not None:
                # deferred: shard i's normalize of the lane's previous step
                # (peaks final: that step's all-reduce ran before on this lane)
                self.b.filter_normalize_prev(xw, lo, hi, n, self.nch, yw, sh.start, sh.end, peaks, sh.file,
                                             pend[0][i], sh.end - sh.start, pend[1], self._slot(sh),
                                             self.normalize)
            elif self.fuse and prev is not None:
                psh, pyw = prev
                self.b.filter_normalize_prev(xw, lo, hi, n, self.nch, yw, sh.start, sh.end, peaks, sh.file,
                                             pyw, psh.end - psh.start, peaks, psh.file, self.normalize)
            else:
                self.b.filter(xw, lo, hi, n, self.nch, yw, sh.start, sh.end, peaks, sh.file)
            prev = (sh, yw)
        if self.exchange:
            self.allreduce_max(peaks)
        if self.defer:
            self._pending[lane] = (outputs, peaks)
            self.b.zero_peaks(nxt)
        else:
            last = len(self.shards) - 1
            for i, (sh, yw) in enumerate(zip(self.shards, outputs)):
                if self.fuse and i < last:
                    continue  # rescaled inside the next shard's filter launch
                if i == last:
                    self.b.normalize_clear(yw, self.nch, sh.end - sh.start, peaks, self._slot(sh),
                                           self.normalize, nxt)
                else:
                    self.b.normalize(yw, self.nch, sh.end - sh.start, peaks, self._slot(sh), self.normalize)
            if not self.shards:
                self.b.zero_peaks(nxt)
        self.peaks = peaks
        self.outputs = outputs
        self._steps[lane] = k + 1
        self._last = lane
        self._lane = (lane + 1) % self.lanes
        if lane != 0:
            self.b.set_lane(0)  # the caller's stream is current again after every step

    def flush(self):
        """Run the normalizes still pending (defer: each lane's last step) as
        passes of their own, on their lanes."""
        for lane, pend in enumerate(self._pending):
            if pend is None:
                continue
            self.b.set_lane(lane)
            for sh, yw in zip(self.shards, pend[0]):
                self.b.normalize(yw, self.nch, sh.end - sh.start, pend[1], self._slot(sh), self.normalize)
            self._pending[lane] = None
        self.b.set_lane(0)

    def results(self):
        """[(shard, output handle)] of the latest step.  The caller's current
        stream is made to wait for that step's lane first, so reading the
        handles there (a copy to the host, a follow-on kernel) needs no
        device-wide synchronisation.  Pending (deferred) normalizes run first."""
        self.flush()
        self.b.publish(self._last)
        return list(zip(self.shards, self.outputs))

    def close(self):
        """Order every lane's outstanding work before the caller's later work
        (and before the runner's buffers can be reused)."""
        self.flush()
        self.b.join_lanes()
        for lane in range(self.lanes):
            self.b.publish(lane)


class DeviceBackend(Backend):
    """gfx950 kernels through the C ABI on torch-allocated HBM: lane 0 is the
    caller's current stream, lanes 1.. are streams of their own."""

    def __init__(self, flt, device, lanes: int = 1, own_streams: bool = False):
        import torch
        import lcfir
        self.torch, self.lc, self.flt, self.dev = torch, lcfir, flt, device
        # own_streams: lane 0 too gets a stream of its own (HIP graph capture
        # cannot run on the default stream; GraphedSteps); it is the current
        # stream after every step
        # the caller's stream at construction: buffers the runner allocates
        # are allocated on it (retain, publish)
        self.alloc_stream = torch.cuda.current_stream(device)
        self.streams = [torch.cuda.Stream(device) if own_streams else self.alloc_stream]
        self.streams += [torch.cuda.Stream(device) for _ in range(lanes - 1)]
        self.stream = self.streams[0]
        self.sp = self.stream.cuda_stream
        # one-graph replays (GraphedSteps.replay) run every lane's steps on
        # lane 0's stream: `dirty` = lanes given eager work since the last
        # replay (the replay waits for them), `graph_waiters` = lanes whose
        # next eager work must wait for the last replay.  Both waits are taken
        # lazily, only for lanes that actually mix eager and replayed steps
        # (each wait costs host time a launch-bound replay cannot spare).
        self.dirty = set()
        self.graph_waiters = set()

    def _after_graph(self, lane):
        # the lane's work of the last one-graph replay ran on lane 0's stream
        if lane in self.graph_waiters:
            self.graph_waiters.discard(lane)
            self.streams[lane].wait_stream(self.streams[0])

    def set_lane(self, lane):
        s = self.streams[lane]
        self._after_graph(lane)
        self.dirty.add(lane)
        self.stream, self.sp = s, s.cuda_stream
        # torch-side work of the step (the RCCL peak exchange) follows the lane
        self.torch.cuda.set_stream(s)

    def join_lanes(self):
        for s in self.streams:
            for o in self.streams:
                if o is not s:
                    s.wait_stream(o)
        self.graph_waiters.clear()  # every lane now follows lane 0's stream too

    def retain(self, handle, lane):
        # allocated on the caller's stream, written/read on another lane's
        # stream (lanes 1.., and lane 0 too with own_streams): the caching
        # allocator must not hand the block out again before that lane's work
        # is done
        if self.streams[lane] != self.alloc_stream:
            handle.record_stream(self.streams[lane])

    def publish(self, lane):
        # the current stream (lane 0's after a step) and the allocation stream
        # both wait for the lane (and, after a one-graph replay, for the
        # graph, which ran the lane's steps on lane 0's stream)
        self._after_graph(lane)
        cur = self.torch.cuda.current_stream(self.dev)
        cur.wait_stream(self.streams[lane])
        if self.alloc_stream != cur:
            self.alloc_stream.wait_stream(self.streams[lane])

    def new_peaks(self, nfiles):
        return self.torch.zeros(max(1, nfiles), dtype=self.torch.float32, device=self.dev)

    def upload(self, file, xw, x_lo, x_hi):
        t = self.torch
        return t.as_tensor(xw, dtype=t.float32).contiguous().to(self.dev)

    def alloc_out(self, nch, count):
        return self.torch.empty((nch, count), dtype=self.torch.float32, device=self.dev)

    def window(self, n, start, end, half):
        # the whole segments the FFT's units read: a split file's outputs are
        # then bit-identical to the unsplit file's (lcfir_ctx_window)
        return self.flt.window(n, start, end)

    def zero_peaks(self, peaks):
        self.lc.peak_reset_dev(peaks, peaks.numel(), self.sp)

    def filter(self, xw, x_lo, x_hi, n, nch, yw, start, end, peaks, slot):
        # every channel's max|y| is folded into the file's slot inside the kernel
        self.flt.filter_window_dev(xw, x_lo, x_hi, xw.shape[1], n, nch, yw, start, yw.shape[1],
                                   start, end, peaks[slot:slot + 1], self.sp, peak_stride=0)

    def normalize(self, yw, nch, count, peaks, slot, force):
        p = peaks if slot is None else peaks[slot:slot + 1]
        self.lc.normalize_dev(yw, yw.shape[1], nch, count, p, p.numel(), force, self.sp)

    def filter_normalize_prev(self, xw, x_lo, x_hi, n, nch, yw, start, end, peaks, slot,
                              prev_yw, prev_count, prev_peaks, prev_slot, force):
        if not prev_yw.is_contiguous() or prev_yw.shape[1] != prev_count:
            return super().filter_normalize_prev(xw, x_lo, x_hi, n, nch, yw, start, end, peaks, slot,
                                                 prev_yw, prev_count, prev_peaks, prev_slot, force)
        pp = prev_peaks if prev_slot is None else prev_peaks[prev_slot:prev_slot + 1]
        self.flt.filter_window_norm_dev(xw, x_lo, x_hi, xw.shape[1], n, nch, yw, start, yw.shape[1],
                                        start, end, peaks[slot:slot + 1], 0, prev_yw,
                                        prev_yw.numel(), pp, pp.numel(), force, self.sp)

    def normalize_clear(self, yw, nch, count, peaks, slot, force, clear):
        p = peaks if slot is None else peaks[slot:slot + 1]
        self.lc.normalize_clear_dev(yw, yw.shape[1], nch, count, p, p.numel(), force, clear,
                                    clear.numel(), self.sp)


class GraphedSteps:
    """BatchRunner steps replayed from captured HIP graphs, for launch-bound
    batches (config 1: 48 000 samples, three launches of a few microseconds
    per step, where host-side issue sets the rate).  Each lane's two next
    steps are captured on that lane's stream, so the lane's peak vectors
    alternate exactly as in eager steps and a replay leaves the runner's
    buffers as the eager steps would: replay() == 2 x lanes step()s (the
    lanes' steps touch disjoint buffers, so their order across lanes does not
    change a byte).  per_lane=False (default) captures all of them into one
    graph, the lanes forked from lane 0's stream; per_lane=True keeps one
    graph per lane, replayed on the lanes' own streams (config 1: 2.53 against
    3.24 Gs/s for one graph at 10 lanes -- each graph launch costs host time).
    Needs a DeviceBackend with own_streams=True and no collective in the step."""

    def __init__(self, runner, backend, per_lane: bool = False):
        torch = backend.torch
        if runner.exchange:
            raise ValueError("a step with a peak exchange (collective) is not captured")
        s0 = backend.streams[0]
        if s0 == torch.cuda.default_stream(backend.dev):
            raise ValueError("lane 0 must be a stream of its own: DeviceBackend(own_streams=True)")
        # eager steps up to a round boundary (the capture starts on lane 0), and
        # at least one on every lane: a partitioned filter's partial-sum scratch
        # is sized per stream by an eager call (lcfir refuses to allocate it
        # inside a capture, where the graph would keep a pointer it does not own)
        while runner._lane != 0 or min(runner._steps) == 0:
            runner.step()
        self.runner, self.backend = runner, backend
        self.per_replay = 2 * runner.lanes
        torch.cuda.synchronize(backend.dev)
        self.graphs = []
        if per_lane:
            for lane, s in enumerate(backend.streams):
                g = torch.cuda.CUDAGraph()
                with torch.cuda.graph(g, stream=s):
                    for _ in range(2):
                        runner._lane = lane
                        runner.step()
                    torch.cuda.set_stream(s)  # step() ends on lane 0; the capture ends on s
                self.graphs.append((s, g))
            runner._lane = 0  # as after 2 x lanes eager steps from lane 0
        else:
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g, stream=s0):
                for s in backend.streams[1:]:
                    s.wait_stream(s0)
                for _ in range(self.per_replay):
                    runner.step()
                for s in backend.streams[1:]:
                    s0.wait_stream(s)
            self.graphs.append((s0, g))
        runner._last = runner.lanes - 1

    def replay(self):
        """Run per_replay steps, each graph on its lane's stream (the caller
        syncs).  One-graph mode: the graph is launched on lane 0's stream but
        runs every lane's steps, so lane 0 first waits for eager work queued
        on the other lanes since the last replay (DeviceBackend.dirty), and
        each other lane's next eager step waits for the graph
        (DeviceBackend.graph_waiters, taken in set_lane): eager steps before
        and after a replay stay in order on every lane, and back-to-back
        replays pay no waits."""
        torch = self.backend.torch
        b = self.backend
        one = len(self.graphs) == 1 and len(b.streams) > 1
        s0 = b.streams[0]
        if one:
            for lane in sorted(b.dirty - {0}):
                s0.wait_stream(b.streams[lane])
            b.dirty.clear()
        for s, g in self.graphs:
            with torch.cuda.stream(s):
                g.replay()
        if one:
            b.graph_waiters = set(range(1, len(b.streams)))


def torch_allreduce_max(group=None):
    """MAX all-reduce over torch.distributed (RCCL for device tensors, gloo on CPU)."""
    import torch.distributed as dist

    def f(peaks):
        dist.all_reduce(peaks, op=dist.ReduceOp.MAX, group=group)
    return f
