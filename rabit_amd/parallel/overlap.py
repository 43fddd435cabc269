"""Gradient allreduce overlapped with the backward pass.

rabit's engine is per host thread (one engine per thread, as in the reference:
`src/engine.cc:29-40`) and a fault-tolerant collective returns only once its result is known
good: the host waits for the device op before the sequence number advances.  Called from the
training thread, every bucket allreduce therefore stalls the thread that enqueues the rest of
the backward pass, and the GPU runs communication and computation one after the other.

`CommThread` moves the engine onto a dedicated host thread.  `OverlappedBuckets` starts each
gradient bucket's allreduce from a backward hook as soon as the bucket is complete: the comm
thread orders it after the bucket's last gradient kernel (a HIP event), runs it on its own HIP
stream, and waits for it there, while the training thread keeps enqueueing the backward kernels
of the earlier layers.  RCCL / the direct transport then move bucket k over xGMI while the GEMMs
of the layers before it run.  `finish()` joins all bucket ops and orders the optimizer step
after them.

Every rabit call of the job (init, checkpoints, collectives, finalize) has to go through the
comm thread: another thread would reach a different, uninitialised engine.

    comm = CommThread(lambda: rabit.init(args, lib="standard", rabit_device=gpu), device=gpu)
    version, state = comm.call(rabit.load_checkpoint)
    buckets = OverlappedBuckets(model.parameters(), comm, bucket_mb=25)
    for step in ...:
        buckets.zero_grad()
        loss = loss_fn(model(x), y)
        loss.backward()          # bucket allreduces start from inside backward
        buckets.finish()         # wait for them; the optimizer runs after
        opt.step()
        comm.call(rabit.checkpoint, state)
    comm.close()                 # rabit.finalize on the comm thread

Fault tolerance is unchanged: the ops are the same `allreduce_prepared` calls in the same order
on every rank (buckets complete in the same order), so a restarted worker replays them.
"""
from __future__ import annotations

import queue
import threading
from concurrent.futures import Future
from typing import Any, Callable, List, Optional

from .. import core as rabit
from .data_parallel import GradientBuckets


class CommThread:
    """A host thread that owns the rabit engine and runs submitted calls in order."""

    def __init__(self, init_fn: Callable[[], Any], device: Optional[int] = None):
        self.device = device
        self._q: "queue.Queue" = queue.Queue()
        self._stream = None
        self._thread = threading.Thread(target=self._loop, name="rabit-comm", daemon=True)
        self._thread.start()
        self.call(init_fn)

    @property
    def stream(self):
        """the HIP stream the comm thread's device collectives run on"""
        return self._stream

    def _loop(self):
        try:
            import torch

            if self.device is not None and torch.cuda.is_available():
                torch.cuda.set_device(self.device)
                self._stream = torch.cuda.Stream()
        except ImportError:
            torch = None
        while True:
            item = self._q.get()
            if item is None:
                return
            fut, fn, args, kwargs, ready = item
            if not fut.set_running_or_notify_cancel():
                continue
            try:
                if self._stream is not None:
                    with torch.cuda.stream(self._stream):
                        if ready is not None:
                            self._stream.wait_event(ready)  # after the submitter's work
                        res = fn(*args, **kwargs)
                        done = torch.cuda.Event()
                        done.record(self._stream)
                        fut.done_event = done
                else:
                    res = fn(*args, **kwargs)
                fut.set_result(res)
            except BaseException as e:  # noqa: BLE001 - handed to the caller
                fut.set_exception(e)

    def submit(self, fn: Callable, *args, **kwargs) -> Future:
        """Run fn on the comm thread after everything the calling thread has enqueued on its
        current HIP stream so far (an event orders the comm stream after it).  The future's
        `done_event` marks the end of fn's device work on the comm stream."""
        fut: Future = Future()
        fut.done_event = None
        ready = None
        if self._stream is not None:
            import torch

            ready = torch.cuda.Event()
            ready.record(torch.cuda.current_stream())
        self._q.put((fut, fn, args, kwargs, ready))
        return fut

    def call(self, fn: Callable, *args, **kwargs) -> Any:
        """submit and wait; the calling thread's stream is ordered after fn's device work"""
        fut = self.submit(fn, *args, **kwargs)
        res = fut.result()
        if fut.done_event is not None:
            import torch

            torch.cuda.current_stream().wait_event(fut.done_event)
        return res

    def close(self, finalize: bool = True):
        if finalize:
            self.call(rabit.finalize)
        self._q.put(None)
        self._thread.join()


class OverlappedBuckets(GradientBuckets):
    """GradientBuckets whose allreduces start during `loss.backward()` on the comm thread.

    Buckets are filled in reverse parameter order (the order backward produces gradients), so
    the bucket of the last layers is complete, and on its way over xGMI, first."""

    def __init__(self, params, comm: CommThread, bucket_mb: float = 25.0, average: bool = True):
        import torch

        plist = [p for p in params if p.requires_grad]
        super().__init__(list(reversed(plist)), bucket_mb=bucket_mb, average=average)
        self.comm = comm
        self._futures: List[Future] = []
        self._pending = [len(g) for g in self._groups]
        where = {}
        for b, group in enumerate(self._groups):
            for p in group:
                where[id(p)] = b
        for p in self.params:
            p.register_post_accumulate_grad_hook(self._make_hook(where[id(p)]))
        self._torch = torch

    def _make_hook(self, b: int):
        def hook(_param):
            self._pending[b] -= 1
            if self._pending[b] == 0:
                self._launch(b)
        return hook

    def _launch(self, b: int):
        bucket = self.buckets[b]
        world = rabit.get_world_size
        average = self.average

        def run():
            # (submit orders this after the hook thread's stream: the bucket's last gradient)
            n = world()
            if bucket.is_cuda and average and n > 1:
                rabit.allreduce_prepared(bucket, bucket, rabit.SUM, rabit.PREP_SCALE, 1.0 / n)
            else:
                rabit.allreduce(bucket, rabit.SUM)
                if average and n > 1:
                    bucket.mul_(1.0 / n)

        self._futures.append(self.comm.submit(run))

    def reduce(self, op: int = rabit.SUM):
        raise RuntimeError("OverlappedBuckets reduce during backward; call finish()")

    def finish(self):
        """Wait for every bucket allreduce of this step; the caller's stream is ordered after
        them (the optimizer step can follow).  Buckets whose hooks did not fire (parameters
        without gradients this step) are reduced here, in bucket order."""
        torch = self._torch
        for b, left in enumerate(self._pending):
            if left > 0:
                self._launch(b)
        for fut in self._futures:
            fut.result()
            if fut.done_event is not None:
                torch.cuda.current_stream().wait_event(fut.done_event)
        self._futures = []
        self._pending = [len(g) for g in self._groups]
        return self.buckets
