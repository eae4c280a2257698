"""The overlapped forward schedule: GeoT of every micro-batch on one HIP stream, the pair tensors
(construct_interact_tensor, deepinteract_utils.py:158-172) of the micro-batches already computed on a
device-queue kernel beside it (include/deepinteract_amd.h, "pair-tensor queue").

Per micro-batch ("job" j, numbered across steps):

    GeoT stream:  [di_pair_help(jobs whose hT slot is about to be reused)]     every `help_every` jobs
                  embed + InitEdge, edge layer, node layer, ..., final node layer -> hT ring[j % ring]
                  (job j - 1 is signalled by the first of these launches, at its start: the kernel
                  boundary after job j - 1's final node layer has released its hT -- no signal launch)
    pair stream:  ONE di_pair_stream launch per step over the step's jobs: its waves wait on the
                  device for each job's signal and take the job's items from the queue

No host event sits between the two streams: the hand-off is a device-side signal word, and the
GeoT stream's only dependency on the pair stream is the help launch that guarantees a ring slot's
previous job is done before the slot is rewritten -- which also stores pair items at the full-chip
rate whenever GeoT has run `ring` jobs ahead. finish() drains every job (the end of a run).
Correctness never depends on the two streams running concurrently (a stream wave that waits longer
than `patience_ms` gives up and the help launches complete the job).

Hardware queues (round 6). The persistent pair-stream launch is issued BEFORE the GeoT launches that
signal its jobs, so it only overlaps them when the two streams reach the GPU through different
hardware queues. HIP multiplexes a process's streams onto GPU_MAX_HW_QUEUES (4 on the box) in-order
queues per priority, least-used first, so an ordinary stream's queue depends on every stream created
before it: in a process with an RCCL communicator (bench.py under torchrun, or --dist) torch's pool
stream landed on the NULL stream's queue, the pair launch sat in front of the GeoT launches and every
stream wave waited out its patience (round 5: 3767 complexes/s, gave_up 1024). The schedule therefore
runs on `schedule_streams(device)`: two streams created with a CU mask covering every CU, which the HIP
runtime places on hardware queues of their own (di_stream_create_dedicated), and it measures the
property at construction (di_streams_concurrent). If two given streams do not run concurrently the
schedule does not launch the pair stream at all (no wave can wait behind its own producer): every job
is completed by a help launch right after its forward ("ordered" mode, the serial rate).
"""
from __future__ import annotations

import atexit
import ctypes

import torch

from . import _lib
from .engine import _Ticker, _ptr, check_on

_DI_DT = {torch.bfloat16: _lib.DI_BF16, torch.float32: _lib.DI_F32}


class PairQueue:
    """Device state of a pair-tensor queue (counters of `capacity` jobs) and its job table."""

    def __init__(self, device, capacity: int):
        self.lib = _lib.load()
        self.device = device
        self.capacity = int(capacity)
        nbytes = self.lib.di_pair_queue_bytes(self.capacity)
        if nbytes <= 0:
            raise ValueError(f"pair queue capacity {capacity}")
        self.state = torch.zeros(nbytes // 4, dtype=torch.int32, device=device)
        self.jobs = torch.zeros(self.capacity * ctypes.sizeof(_lib.DiPairJob), dtype=torch.uint8, device=device)

    def set_jobs(self, jobs):
        """jobs: sequence of _lib.DiPairJob (device pointers inside), indexed by job number."""
        if len(jobs) > self.capacity:
            raise ValueError("more jobs than the queue holds")
        arr = (_lib.DiPairJob * len(jobs))(*jobs)
        host = torch.frombuffer(bytearray(bytes(arr)), dtype=torch.uint8)
        self.jobs[:host.numel()].copy_(host)

    def reset(self):
        self.state.zero_()

    def counters(self) -> dict:
        """Host copy of the queue's counters (synchronises with the device)."""
        s = self.state[:64].cpu()
        u64 = lambda i: (int(s[i]) & 0xffffffff) | ((int(s[i + 1]) & 0xffffffff) << 32)  # noqa: E731
        return {"signalled": int(s[_lib.PQ_READY]) & 0xffffffff, "error": int(s[_lib.PQ_ERROR]) & 0xffffffff,
                "gave_up": int(s[_lib.PQ_GAVE_UP]) & 0xffffffff, "stream_bytes": u64(_lib.PQ_SBYTES),
                "help_bytes": u64(_lib.PQ_HBYTES)}


_STREAMS = {}


def _destroy_streams():
    """atexit: drain and destroy the dedicated streams while the HIP runtime is still up (left to the
    runtime's own teardown they crashed the process at exit under rocprofv3)."""
    if not _STREAMS:
        return
    lib = _lib.load()
    for idx, pair in list(_STREAMS.items()):
        try:
            torch.cuda.synchronize(idx)
        except RuntimeError:
            pass
        for st in pair:
            lib.di_stream_destroy(ctypes.c_void_p(st.cuda_stream))
    _STREAMS.clear()


def schedule_streams(device=None):
    """(GeoT stream, pair stream) of the overlapped schedule on `device`: two torch ExternalStreams on
    hardware queues of their own (di_stream_create_dedicated), created once per process and device and
    shared by every schedule. Nothing else should be issued on the NULL stream while a step runs (the
    streams are blocking streams)."""
    dev = torch.device(device if device is not None else "cuda")
    idx = dev.index if dev.index is not None else torch.cuda.current_device()
    if idx not in _STREAMS:
        lib = _lib.load()
        if not _STREAMS:
            atexit.register(_destroy_streams)
        handles = []
        with torch.cuda.device(idx):
            for _ in range(2):
                h = ctypes.c_void_p()
                _lib.check(lib.di_stream_create_dedicated(ctypes.byref(h)), "di_stream_create_dedicated")
                handles.append(h.value)
        _STREAMS[idx] = tuple(torch.cuda.ExternalStream(h, device=torch.device("cuda", idx)) for h in handles)
    return _STREAMS[idx]


def streams_concurrent(a, b, patience_ms: float = 200.0) -> bool:
    """Whether work issued on stream b runs while a kernel issued earlier on stream a is still running
    (di_streams_concurrent: the two streams are on different hardware queues). Synchronises both."""
    lib = _lib.load()
    work = torch.zeros(64, dtype=torch.int32, device=a.device)
    torch.cuda.synchronize(a.device)
    out = ctypes.c_int32(-1)
    _lib.check(lib.di_streams_concurrent(ctypes.c_void_p(a.cuda_stream), ctypes.c_void_p(b.cuda_stream), _ptr(work),
                                         float(patience_ms), ctypes.byref(out)), "di_streams_concurrent")
    return out.value == 1


class OverlappedSchedule:
    """GeoT || pair tensor over resident micro-batches (graph batches of equal shape).

    eng: GeoTEngine; mbs: list of GraphBatch (one step = every micro-batch once); h1r/h2r/l1/l2: the
    per-complex pair descriptors (rows in the micro-batch, chain lengths), the same for every
    micro-batch; sinks: output buffers, job j writes sinks[j % len(sinks)] (a list with one buffer per
    job keeps every pair tensor). Up to `ring` jobs are in flight, so with fewer than `ring` sinks two
    jobs in flight may write one buffer at once: that needs discard_outputs=True (a benchmark that never
    reads them). s_geot / s_pair: the two HIP streams (None: schedule_streams(device), the default);
    streams that turn out not to run concurrently put the schedule in "ordered" mode (module doc).
    tap(job, h, e): called right after each micro-batch's forward is issued, with the engine's node /
    edge feature outputs of that forward, while the GeoT stream is current (stream-ordered copies taken
    there see exactly what the schedule computed, before the workspace is reused)."""

    def __init__(self, eng, mbs, h1r, h2r, l1, l2, sinks, s_geot=None, s_pair=None, ring=16, help_every=4,
                 stream_blocks=0, stream_waves=0, help_blocks=0, help_waves=0, patience_ms=20.0,
                 capacity_steps=64, jobs_per_launch=0, discard_outputs=False, tap=None):
        if help_every < 1 or ring < 2 * help_every:
            raise ValueError("need ring >= 2 * help_every")
        if eng.dtype == "bf16" and not eng.fuse_embed_init and eng.resident_init:
            # its 12-wave block (3 x 168 VGPRs per SIMD) does not fit on a SIMD holding a pair-stream
            # wave, and the default pair launch puts store waves on every CU: InitEdge would wait for
            # the pair waves to give up (measured: gave_up on every wave)
            raise ValueError("the LDS-resident InitEdge (engine.resident_init) cannot run beside the pair "
                             "stream: set eng.resident_init = False or keep eng.fuse_embed_init")
        self.eng, self.mbs = eng, mbs
        if s_geot is None or s_pair is None:
            g, p = schedule_streams(eng.device)
            s_geot, s_pair = s_geot or g, s_pair or p
        self.s_geot, self.s_pair = s_geot, s_pair
        self.tap, self.discard_outputs = tap, bool(discard_outputs)
        # the property the persistent pair launch needs (module doc); measured, not assumed
        self.concurrent = s_geot is not s_pair and streams_concurrent(s_pair, s_geot)
        self.mode = "overlapped" if self.concurrent else "ordered"
        self.ring, self.help_every, self.patience = ring, help_every, float(patience_ms)
        # pair-stream launches cover this many jobs each (0: one launch per step)
        self.jobs_per_launch = int(jobs_per_launch) or len(mbs)
        dev = eng.device
        dt = torch.bfloat16 if eng.dtype == "bf16" else torch.float32
        self.dt, self.di_dt = dt, _DI_DT[dt]
        H = eng.cfg.num_gnn_hidden_channels
        self.hidden = H
        self.l1, self.l2 = list(l1), list(l2)
        n_rows = mbs[0].num_nodes
        if any(gb.num_nodes != n_rows for gb in mbs):
            raise ValueError("the micro-batches of a schedule must have equal node counts (one hT ring)")
        vec = 16 // torch.tensor([], dtype=dt).element_size()
        if n_rows % vec or any(l % vec for l in l2) or any(r % vec for r in h2r):
            raise ValueError("the pair queue needs 16-B aligned planes (L2, h2 rows multiples of 16 B)")
        self.hT = [torch.empty(H, n_rows, dtype=dt, device=dev) for _ in range(ring)]
        descs = (_lib.DiPairDesc * len(l1))()
        off, self.offs = 0, []
        for i, (a, b, x, y) in enumerate(zip(h1r, h2r, l1, l2)):
            descs[i] = _lib.DiPairDesc(a, b, off, x, y)
            self.offs.append(off)
            off += 2 * H * x * y
        self.numel = off
        self.descs = torch.frombuffer(bytearray(bytes(descs)), dtype=torch.uint8).to(dev)
        for s in sinks:
            check_on(dev, "OverlappedSchedule", s)
            if s.dtype != dt or s.numel() < off or s.data_ptr() % 16:
                raise ValueError("pair sink: wrong dtype, too small or not 16-B aligned")
        self.sinks = sinks
        self.items = eng.lib.di_pair_job_items(len(l1), max(l1), H)
        if self.items <= 0:
            raise ValueError("pair job too large")
        self.queue = PairQueue(dev, capacity_steps * len(mbs))
        jobs = [_lib.DiPairJob(self.hT[j % ring].data_ptr(), self.descs.data_ptr(), sinks[j % len(sinks)].data_ptr(),
                               n_rows, len(l1), max(l1), self.items) for j in range(self.queue.capacity)]
        self.queue.set_jobs(jobs)
        self.stream_launch = _lib.DiPairLaunch(_lib.DI_PAIR_ROWS, int(stream_blocks), int(stream_waves), 1)
        self.help_launch = _lib.DiPairLaunch(_lib.DI_PAIR_ROWS, int(help_blocks), int(help_waves), 0)
        self.next_job = 0   # job number of the next micro-batch
        self.helped = 0     # every job below this one is guaranteed complete by an issued help launch
        self.pending = -1   # the last job produced and not yet signalled (carried by the next launch)
        self.help_launches = 0

    # ---- issue helpers -----------------------------------------------------------------------
    def _q(self):
        return _ptr(self.queue.state)

    def _help(self, first, last, st):
        _lib.check(self.eng.lib.di_pair_help(self.di_dt, _ptr(self.queue.jobs), first, last, self.hidden, self._q(),
                                             ctypes.byref(self.help_launch), self.pending, st), "di_pair_help")
        self.pending = -1
        self.help_launches += 1

    def _stream(self, j0, j1, st):
        _lib.check(self.eng.lib.di_pair_stream(self.di_dt, _ptr(self.queue.jobs), j0, j1, self.hidden, self._q(),
                                               ctypes.byref(self.stream_launch), self.patience, st), "di_pair_stream")

    def _rollover(self):
        """Restart job numbering when the queue's counters are used up (drain, sync, zero)."""
        if self.next_job + len(self.mbs) <= self.queue.capacity:
            return
        self.finish()
        torch.cuda.synchronize(self.eng.device)
        self.check()
        self.queue.reset()
        self.next_job = self.helped = 0
        self.pending = -1

    def step(self, events=None, geot_events=None):
        """Issue one step (every micro-batch once). events: HIP event pairs around the pair-stream
        launch (dict key "pair_tensor"); geot_events: around every GeoT launch (per-kernel timing)."""
        self._rollover()
        j0, n = self.next_job, len(self.mbs)
        if len(self.sinks) < self.ring and j0 + n > len(self.sinks) and not self.discard_outputs:
            raise ValueError(f"{len(self.sinks)} sinks for up to {self.ring} jobs in flight: job {len(self.sinks)} "
                             f"would overwrite job 0's pair tensors while it may still be written (pass "
                             f"discard_outputs=True if they are never read)")
        if self.concurrent:
            with torch.cuda.stream(self.s_pair):
                tick = _Ticker(events)
                for a in range(j0, j0 + n, self.jobs_per_launch):
                    tick("pair_tensor")
                    self._stream(a, min(a + self.jobs_per_launch, j0 + n), ctypes.c_void_p(self.s_pair.cuda_stream))
                tick(None)
        with torch.cuda.stream(self.s_geot):
            st = ctypes.c_void_p(self.s_geot.cuda_stream)
            for m, gb in enumerate(self.mbs):
                j = j0 + m
                if self.concurrent and j % self.help_every == 0:
                    # jobs j .. j + help_every - 1 reuse the ring slots of jobs up to j + help_every - 1 - ring
                    last = j + self.help_every - 1 - self.ring
                    if last >= self.helped:
                        self._help(self.helped, last, st)
                        self.helped = last + 1
                # this forward's first launch signals job j - 1 unless a help launch just did
                h, e = self.eng.forward(gb, clone=False, events=geot_events, hT_out=self.hT[j % self.ring],
                                        signal=(self.queue.state, self.pending) if self.pending >= 0 else None)
                if self.tap is not None:
                    self.tap(j, h, e)
                self.pending = j
                if not self.concurrent:
                    # ordered mode: the job's pair tensors by a help launch right behind its forward
                    # (which also signals it); no launch ever waits on the device for a later one
                    tick = _Ticker(events)
                    tick("pair_tensor")
                    self._help(j, j, st)
                    tick(None)
                    self.helped = j + 1
        self.next_job = j0 + n

    def finish(self):
        """Drain: a help launch over every job not yet guaranteed complete (on the GeoT stream)."""
        with torch.cuda.stream(self.s_geot):
            st = ctypes.c_void_p(self.s_geot.cuda_stream)
            if self.helped < self.next_job:
                self._help(self.helped, self.next_job - 1, st)  # carries the last job's signal
                self.helped = self.next_job
            elif self.pending >= 0:
                _lib.check(self.eng.lib.di_pair_signal(self._q(), self.pending, st), "di_pair_signal")
                self.pending = -1

    def check(self, allow_gave_up=False):
        """Host read of the queue's counters (synchronises). Raises if a help launch's completion wait
        timed out or a stream wave read a non-increasing ticket (error word), and -- unless
        allow_gave_up -- if any stream wave gave up waiting for a signal: the outputs are still complete
        then (the help launches wrote them), but the overlap the schedule exists for did not happen."""
        c = self.queue.counters()
        if c["error"]:
            raise RuntimeError(f"pair queue error {c}")
        if c["gave_up"] and not allow_gave_up:
            raise RuntimeError(f"pair stream waves gave up waiting for their signal (the streams did not run "
                               f"concurrently): {c}")
        return c

    def views(self, job, buf=None):
        """The [1, 2H, L1, L2] pair tensors job `job` wrote (valid until its sink is reused, i.e. until
        job + len(sinks) is issued), or the same views of `buf` (a copy of its sink)."""
        out, H = (self.sinks[job % len(self.sinks)] if buf is None else buf), self.hidden
        return [out[o:o + 2 * H * a * b].view(1, 2 * H, a, b) for o, a, b in zip(self.offs, self.l1, self.l2)]
