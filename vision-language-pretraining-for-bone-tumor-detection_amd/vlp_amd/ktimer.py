"""Per-kernel-family HIP event timing on the launch stream (used by bench.py
for the roofline line).  A "family" is one kernel instantiation (= one name in
a rocprofv3 --stats summary), e.g. the 128x128-tile implicit-GEMM forward conv
with BN+ReLU-on-load.  Disabled => one branch per launch."""
from __future__ import annotations

import torch

_ENABLED = False
_ONLY = None
_REC = {}   # key -> list of (start_event, end_event, flops)


def enable(only=None):
    global _ENABLED, _ONLY, _REC
    _ENABLED, _ONLY, _REC = True, only, {}


def disable():
    global _ENABLED
    _ENABLED = False


def begin(key, flops=0.0):
    if not _ENABLED or (_ONLY is not None and key != _ONLY):
        return None
    s = torch.cuda.Event(enable_timing=True)
    e = torch.cuda.Event(enable_timing=True)
    s.record(torch.cuda.current_stream())
    return (key, s, e, flops)


def end(tok):
    if tok is None:
        return
    key, s, e, flops = tok
    e.record(torch.cuda.current_stream())
    _REC.setdefault(key, []).append((s, e, flops))


def totals():
    """key -> (total ms, launches, total flops); call after synchronize()."""
    out = {}
    for k, lst in _REC.items():
        ms = sum(s.elapsed_time(e) for s, e, _ in lst)
        out[k] = (ms, len(lst), sum(f for _, _, f in lst))
    return out
