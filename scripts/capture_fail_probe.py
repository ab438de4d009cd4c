"""What a failure inside torch.cuda.graph leaves behind:
variant raise = an exception inside the capture; malloc = a hipMalloc under
capture, then the exception; malloc_noraise = the hipMalloc alone; *_keep =
the failed CUDAGraph object is kept alive instead of deleted; reset = its
reset() is called explicitly. Prints each step so a terminate shows where."""
import ctypes
import gc
import sys

import torch

variant = sys.argv[1]
hip = ctypes.CDLL("libamdhip64.so.7")
x = torch.zeros(1 << 20, device="cuda")
torch.cuda.synchronize()
g = torch.cuda.CUDAGraph()
fresh = "fresh" in variant   # every capture on a stream of its own
ctx = torch.cuda.graph(g, stream=torch.cuda.Stream()) if fresh else torch.cuda.graph(g)
try:
    with ctx:
        x.add_(1)
        if variant.startswith("malloc"):
            p = ctypes.c_void_p()
            print("hipMalloc under capture rc", hip.hipMalloc(ctypes.byref(p), 1 << 20), flush=True)
        if not variant.startswith("malloc_noraise"):
            raise RuntimeError("hook")
    print("capture ended without exception", flush=True)
except Exception as e:  # noqa: BLE001
    print("caught", type(e).__name__, str(e)[:300].replace("\n", " | "), flush=True)
st = ctypes.c_int(-1)
hip.hipStreamIsCapturing(ctypes.c_void_p(ctx.capture_stream.cuda_stream), ctypes.byref(st))
print("capture status", st.value, "current", torch.cuda.current_stream(), "default",
      torch.cuda.default_stream(), flush=True)
if st.value and not fresh:
    gr = ctypes.c_void_p()
    print("end capture rc", hip.hipStreamEndCapture(ctypes.c_void_p(ctx.capture_stream.cuda_stream),
                                                   ctypes.byref(gr)), flush=True)
torch.cuda.set_stream(torch.cuda.default_stream())
print("last error", hip.hipGetLastError(), flush=True)
if "reset" in variant:
    try:
        g.reset()
        print("reset ok", flush=True)
    except Exception as e:  # noqa: BLE001
        print("reset raised", str(e)[:200].replace("\n", " | "), flush=True)
if "keep" in variant:
    KEEP = g
else:
    del g
    gc.collect()
    print("deleted the graph", flush=True)
x.add_(1)
torch.cuda.synchronize()
print("eager ok", x[0].item(), flush=True)
y = torch.empty(1 << 28, device="cuda")   # a fresh hipMalloc after the failure
y.fill_(1)
torch.cuda.synchronize()
print("allocation after the failure ok", flush=True)
g2 = torch.cuda.CUDAGraph()
with (torch.cuda.graph(g2, stream=torch.cuda.Stream()) if fresh else torch.cuda.graph(g2)):
    x.add_(1)
g2.replay()
torch.cuda.synchronize()
print("second capture ok", x[0].item(), flush=True)
