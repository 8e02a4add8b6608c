"""Step watchdog: hang forensics without re-running (bench.py).

When armed, every `_lib.call` entry point records its name on the HIP stream it is launched on,
followed by a (non-timing) HIP event, in a short per-stream ring; optionally (`ops=True`) a
TorchDispatchMode records the torch-level ops enqueued per stream the same way (autograd's
device thread inherits the mode, so backward ops are seen too). A monitor thread watches the
step-end events: when a step has been pending for longer than `factor` x the median completed
step (never less than `floor_s`), it writes a report -- per stream the last markers with whether
each has completed on the device, so the first pending marker names the work in flight; the
Python stacks of every thread -- and ends the process with a non-zero status (`os._exit`, no
re-exec). One process, no GPU work of its own: the report only queries events.
"""
from __future__ import annotations

import collections
import faulthandler
import json
import os
import statistics
import threading
import time

import torch

from . import _lib

RING = 48


class _OpMode(torch.utils._python_dispatch.TorchDispatchMode):
    def __init__(self, wd):
        super().__init__()
        self.wd = wd

    def __torch_dispatch__(self, func, types, args=(), kwargs=None):
        out = func(*args, **(kwargs or {}))
        self.wd.note("op:" + str(func.overloadpacket.__name__), event=False)
        return out


class StepWatchdog:
    def __init__(self, device, out_path, factor=10.0, floor_s=20.0, first_floor_s=240.0, ops=False, poll_s=0.25):
        self.device = torch.device(device)
        self.out_path = out_path
        self.factor, self.floor_s, self.first_floor_s, self.poll_s = factor, floor_s, first_floor_s, poll_s
        self.rings = collections.defaultdict(lambda: collections.deque(maxlen=RING))
        self.ops_rings = collections.defaultdict(lambda: collections.deque(maxlen=RING))
        self.lock = threading.Lock()
        self.pending = collections.deque()     # (step index, end event, host time enqueued)
        self.durations = []
        self.step_idx = 0
        self.last_done_t = None
        self._stop = threading.Event()
        self._mode = _OpMode(self) if ops else None
        self._thread = None

    # -- recording ------------------------------------------------------------------------
    def note(self, name, event=True):
        s = torch.cuda.current_stream(self.device)
        ev = None
        if event:
            ev = torch.cuda.Event()
            ev.record(s)
        with self.lock:
            (self.rings if event else self.ops_rings)[s.cuda_stream].append((name, ev, time.monotonic()))

    def step_begin(self):
        if self.last_done_t is None:
            self.last_done_t = time.monotonic()

    def step_end(self):
        ev = torch.cuda.Event()
        ev.record(torch.cuda.current_stream(self.device))
        with self.lock:
            self.pending.append((self.step_idx, ev, time.monotonic()))
        self.step_idx += 1

    # -- control --------------------------------------------------------------------------
    def __enter__(self):
        _lib.WATCH = self
        if self._mode is not None:
            self._mode.__enter__()
        self._thread = threading.Thread(target=self._monitor, name="triad-step-watchdog", daemon=True)
        self._thread.start()
        return self

    def __exit__(self, *exc):
        if self._mode is not None:
            self._mode.__exit__(*exc)
        _lib.WATCH = None
        self._stop.set()
        if self._thread is not None:
            self._thread.join(timeout=5)
        return False

    def _limit(self):
        if not self.durations:
            return self.first_floor_s
        return max(self.floor_s, self.factor * statistics.median(self.durations))

    def _monitor(self):
        while not self._stop.wait(self.poll_s):
            now = time.monotonic()
            with self.lock:
                while self.pending and self.pending[0][1].query():
                    self.pending.popleft()
                    if self.last_done_t is not None:
                        self.durations.append(now - self.last_done_t)
                    self.last_done_t = now
                head = self.pending[0] if self.pending else None
            if head is None or self.last_done_t is None:
                continue
            # the stalled step could not start on the device before the previous one ended, nor
            # before the host enqueued it
            waited = now - max(self.last_done_t, head[2])
            if waited > self._limit():
                self._report(head[0], waited)
                os._exit(3)

    def _report(self, step, waited):
        rep = {"stalled_step": step, "waited_s": round(waited, 1), "limit_s": round(self._limit(), 1),
               "median_step_s": statistics.median(self.durations) if self.durations else None, "streams": {}}
        with self.lock:
            for sid, ring in self.rings.items():
                rows, first_pending = [], None
                for name, ev, t in ring:
                    done = bool(ev.query())
                    rows.append({"entry": name, "done": done})
                    if not done and first_pending is None:
                        first_pending = name
                rep["streams"][hex(sid)] = {"in_flight_or_next": first_pending,
                                            "last_completed": next((r["entry"] for r in reversed(rows) if r["done"]),
                                                                   None),
                                            "markers": rows,
                                            "last_torch_ops": [n for n, _, _ in self.ops_rings.get(sid, [])]}
        with open(self.out_path, "w") as f:
            json.dump(rep, f, indent=1)
            f.write("\n\n# python stacks of every thread\n")
            f.flush()
            faulthandler.dump_traceback(file=f, all_threads=True)
        print(f"[watchdog] step {step} pending {waited:.0f} s (limit {self._limit():.0f} s): report in "
              f"{self.out_path}", flush=True)


def arm(device, out_path=None, **kw):
    out_path = out_path or os.environ.get("TRIAD_WATCHDOG_OUT", "bench_watchdog.json")
    return StepWatchdog(device, out_path, **kw)
