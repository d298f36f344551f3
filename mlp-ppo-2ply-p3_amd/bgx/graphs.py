"""HIP graph capture of engine steps, and what a failed capture means.

A capture of `Engine.step` / `PolicyNet.act` calls records launches but also
advances the engine's host state (overflow-counter parity, the pending dispatch
order on the side stream; csrc/bg_engine.hip) as if the steps had run.  When a
capture fails part-way, that host state describes steps that never ran, and the
stream may be left in capture mode (round 3, gpurun_out/r3h: an eager fallback
after a failed capture raised hipErrorStreamCaptureImplicit and both ranks then
died with SIGSEGV in teardown).  So a failed capture is terminal: `capture`
prints the error and ends the process with EXIT_CAPTURE_FAILED without running
destructors over a stream that may still be capturing.

BGX_INJECT_CAPTURE_FAILURE=<site> (tests only) makes the capture at that site
fail for real: a stream synchronize inside the capture, which HIP refuses and
which invalidates the capture.
"""
from __future__ import annotations

import gc
import os
import sys

import torch

EXIT_CAPTURE_FAILED = 3


def _inject(site: str):
    if os.environ.get("BGX_INJECT_CAPTURE_FAILURE") == site:
        torch.cuda.current_stream().synchronize()      # illegal while capturing


def capture(site: str, body, stream: torch.cuda.Stream) -> torch.cuda.CUDAGraph:
    """Capture `body()` on `stream` into a new graph (thread-local capture mode,
    so another thread's event queries, e.g. an RCCL watchdog's, cannot invalidate
    it).  On any failure: message on stderr, then os._exit(EXIT_CAPTURE_FAILED)."""
    g = torch.cuda.CUDAGraph()
    # no cyclic garbage collection while capturing: torch.cuda.graph collects before the
    # capture starts, but a collection triggered inside it would run finalizers (stream,
    # event and graph destructors of earlier captures) that HIP refuses mid-capture -- an
    # abort, not an exception (round 6: a recapture inside PPOTrainer.update)
    gc_was = gc.isenabled()
    gc.disable()
    try:
        with torch.cuda.graph(g, stream=stream, capture_error_mode="thread_local"):
            body()
            _inject(site)
    except Exception as ex:                              # noqa: BLE001 - every failure is terminal
        sys.stdout.flush()
        sys.stderr.write(f"bgx: HIP graph capture failed at {site}: {type(ex).__name__}: {ex}\n"
                         "bgx: the engines' host state already advanced through the captured steps and the "
                         "stream may still be capturing; exiting (no eager continuation)\n")
        sys.stderr.flush()
        os._exit(EXIT_CAPTURE_FAILED)
    finally:
        if gc_was:
            gc.enable()
    return g
