#!/usr/bin/env python3
"""Diagnose the HIP state after a stream capture aborted by an exception (GPU box)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from cuda_mpi_reductions_amd._native import native  # noqa: E402

C = native()
dev = torch.device("cuda", 0)
x = torch.ones(3, device=dev)
g = torch.cuda.CUDAGraph()
cap_stream = None
try:
    with torch.cuda.graph(g):
        cap_stream = torch.cuda.current_stream()
        x.add_(1)
        torch.cuda.synchronize()
except Exception as e:
    print("capture raised:", type(e).__name__, str(e).splitlines()[0])
h = cap_stream.cuda_stream
print("capture stream status:", C.stream_capture_status(h))
if "--restore" in sys.argv:
    torch.cuda.set_stream(torch.cuda.default_stream(dev))
print("null stream status:", C.stream_capture_status(0))
print("current stream status:", C.stream_capture_status(torch.cuda.current_stream().cuda_stream))
print("last error:", repr(C.hip_get_last_error()))


def probe(tag):
    try:
        v = torch.ones(3, device=dev).sum().item()
        print(tag, "launch ok", v)
        return True
    except Exception as e:
        print(tag, "launch failed:", str(e).splitlines()[0])
        return False


if not probe("after clear:"):
    print("end_capture(capture stream):", repr(C.end_capture(h)))
    print("capture stream status:", C.stream_capture_status(h))
    print("last error:", repr(C.hip_get_last_error()))
    if not probe("after end_capture:"):
        s = torch.cuda.Stream(dev)
        with torch.cuda.stream(s):
            probe("fresh stream:")
