"""Probe: HIP stream state after a hipGraph capture invalidated by a synchronisation (what
qmc.abandon_capture must handle).  Prints hipStreamIsCapturing (rc, status) per stream."""
import ctypes
import torch

h = ctypes.CDLL("libamdhip64.so")
h.hipStreamIsCapturing.argtypes = [ctypes.c_void_p, ctypes.POINTER(ctypes.c_int)]
h.hipStreamEndCapture.argtypes = [ctypes.c_void_p, ctypes.POINTER(ctypes.c_void_p)]
h.hipGetLastError.restype = ctypes.c_int


def st(name, s):
    v = ctypes.c_int(-9)
    rc = h.hipStreamIsCapturing(ctypes.c_void_p(s.cuda_stream), ctypes.byref(v))
    print("%-8s ptr=%#x rc=%d status=%d" % (name, s.cuda_stream, rc, v.value), flush=True)
    return rc, v.value


x = torch.ones(16, device="cuda")
caller = torch.cuda.current_stream()
s = torch.cuda.Stream()
s.wait_stream(caller)
g = torch.cuda.CUDAGraph()
try:
    with torch.cuda.stream(s):
        with torch.cuda.graph(g, stream=s):
            y = x * 2
            torch.cuda.current_stream().synchronize()
except Exception as e:
    print("capture failed:", type(e).__name__, str(e).splitlines()[0], flush=True)
st("side", s)
st("caller", caller)
st("default", torch.cuda.default_stream())
print("lasterr", h.hipGetLastError(), flush=True)
for name, ss in (("side", s), ("caller", caller)):
    gr = ctypes.c_void_p(None)
    rc = h.hipStreamEndCapture(ctypes.c_void_p(ss.cuda_stream), ctypes.byref(gr))
    print("endcapture", name, rc, gr.value, flush=True)
st("side", s)
st("caller", caller)
print("lasterr", h.hipGetLastError(), flush=True)
try:
    z = (x * 3).sum().item()
    print("eager after failure ok", z, flush=True)
except Exception as e:
    print("eager after failure FAILED", type(e).__name__, str(e).splitlines()[0], flush=True)
try:
    s2 = torch.cuda.Stream()
    with torch.cuda.stream(s2):
        w = (x * 4).sum()
    s2.synchronize()
    print("fresh stream ok", float(w), flush=True)
except Exception as e:
    print("fresh stream FAILED", type(e).__name__, str(e).splitlines()[0], flush=True)
