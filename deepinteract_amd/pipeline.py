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
"""
from __future__ import annotations

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


class OverlappedSchedule:
    """GeoT || pair tensor over resident micro-batches (graph batches of equal shape).

    eng: GeoTEngine; mbs: list of GraphBatch (one step = every micro-batch once); h1r/h2r/l1/l2: the
    per-complex pair descriptors (rows in the micro-batch, chain lengths), the same for every
    micro-batch; sinks: output buffers, job j writes sinks[j % len(sinks)] (a list with one buffer per
    job keeps every pair tensor). s_geot / s_pair: the two HIP streams."""

    def __init__(self, eng, mbs, h1r, h2r, l1, l2, sinks, s_geot, s_pair, ring=16, help_every=4,
                 stream_blocks=0, stream_waves=0, help_blocks=0, help_waves=0, patience_ms=20.0,
                 capacity_steps=64, jobs_per_launch=0):
        if help_every < 1 or ring < 2 * help_every:
            raise ValueError("need ring >= 2 * help_every")
        self.eng, self.mbs = eng, mbs
        self.s_geot, self.s_pair = s_geot, s_pair
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
                if j % self.help_every == 0:
                    # jobs j .. j + help_every - 1 reuse the ring slots of jobs up to j + help_every - 1 - ring
                    last = j + self.help_every - 1 - self.ring
                    if last >= self.helped:
                        self._help(self.helped, last, st)
                        self.helped = last + 1
                # this forward's first launch signals job j - 1 unless a help launch just did
                self.eng.forward(gb, clone=False, events=geot_events, hT_out=self.hT[j % self.ring],
                                 signal=(self.queue.state, self.pending) if self.pending >= 0 else None)
                self.pending = j
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

    def check(self):
        """Raise if a help launch's completion wait timed out (host read of the queue's error word)."""
        c = self.queue.counters()
        if c["error"]:
            raise RuntimeError(f"pair queue error {c}")
        return c

    def views(self, job):
        """The [1, 2H, L1, L2] pair tensors job `job` wrote (valid until its sink is reused)."""
        out, H = self.sinks[job % len(self.sinks)], self.hidden
        return [out[o:o + 2 * H * a * b].view(1, 2 * H, a, b) for o, a, b in zip(self.offs, self.l1, self.l2)]
