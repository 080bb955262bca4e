"""Which HIP call inside a stream capture ends in the round-4 segfault at capture_end?
(gpurun_out/r04g/tests.log, test_graph_capture_forward_backward crashed in
torch.cuda.graphs.capture_end, i.e. in hipStreamEndCapture.)  At that commit a sample backward
under capture issued, besides its kernels, a stream-ordered allocation of the slot sums
(hipMallocAsync + hipFreeAsync on the capturing stream, dgs_sample.hip) -- the calls round 5
removed from the boundary.  One scenario per process, each a torch.cuda.graph capture of a torch
op plus raw HIP calls on the capturing stream through ctypes (the HIP library torch loaded):

    python tools/graph_probe3.py SCENARIO

  plain          torch ops only (control)
  memset         + hipMemsetAsync into a torch-allocated buffer (a kernel-like node)
  malloc_free    + hipMallocAsync, hipMemsetAsync into it, hipFreeAsync, all inside the capture
                   (round 4's slot-sum pattern)
  malloc_only    + hipMallocAsync inside the capture, hipFreeAsync after it
  raise_inside   a Python exception inside the capture (torch.cuda.graph's __exit__ still ends it)
  sync_inside    + hipStreamSynchronize on the capturing stream (illegal under capture: the
                   round-4 library synced there when its call-time tile lists were first built,
                   and then returned an error, raised inside the capture), then the capture ends

Prints "<scenario>: ok (rc of each HIP call)" when the capture ends and the graph replays.
"""
import ctypes
import sys

import torch


def hip_lib():
    """The libamdhip64 mapped into this process by torch (not a second copy from /opt/rocm)."""
    torch.zeros(1, device="cuda")
    for line in open("/proc/self/maps"):
        path = line.split()[-1]
        if "libamdhip64.so" in path:
            return ctypes.CDLL(path)
    return ctypes.CDLL("libamdhip64.so")


def run(scenario):
    hip = hip_lib()
    hip.hipMallocAsync.argtypes = [ctypes.POINTER(ctypes.c_void_p), ctypes.c_size_t, ctypes.c_void_p]
    hip.hipFreeAsync.argtypes = [ctypes.c_void_p, ctypes.c_void_p]
    hip.hipMemsetAsync.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_size_t, ctypes.c_void_p]
    x = torch.randn(1 << 20, device="cuda")
    buf = torch.empty(1 << 20, device="cuda")
    rcs = []
    held = ctypes.c_void_p()
    g = torch.cuda.CUDAGraph()
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        y = x * 2.0  # warm-up of the op outside the capture
    torch.cuda.current_stream().wait_stream(s)
    torch.cuda.synchronize()
    if scenario in ("raise_inside", "sync_inside"):
        try:
            with torch.cuda.graph(g):
                st = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
                y = x * 3.0
                if scenario == "sync_inside":
                    hip.hipStreamSynchronize.argtypes = [ctypes.c_void_p]
                    rcs.append(hip.hipStreamSynchronize(st))
                    print(f"{scenario}: hipStreamSynchronize rc {rcs[-1]}; raising inside the capture", flush=True)
                raise RuntimeError("an error raised inside the capture")
        except Exception as e:  # (what torch.cuda.graph's __exit__ made of it)
            rcs.append(f"{type(e).__name__}: {e}"[:200])
        print(f"{scenario}: ok, the capture ended without a crash (rc {rcs})", flush=True)
        return
    with torch.cuda.graph(g):
        st = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
        y = x * 2.0
        if scenario == "memset":
            rcs.append(hip.hipMemsetAsync(ctypes.c_void_p(buf.data_ptr()), 0, buf.numel() * 4, st))
        elif scenario in ("malloc_free", "malloc_only"):
            rcs.append(hip.hipMallocAsync(ctypes.byref(held), 1 << 22, st))
            rcs.append(hip.hipMemsetAsync(held, 0, 1 << 22, st))
            if scenario == "malloc_free":
                rcs.append(hip.hipFreeAsync(held, st))
        print(f"{scenario}: calls issued, rc {rcs}; ending the capture", flush=True)
    print(f"{scenario}: capture ended", flush=True)
    g.replay()
    torch.cuda.synchronize()
    if scenario == "malloc_only":
        rcs.append(hip.hipFreeAsync(held, ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)))
        torch.cuda.synchronize()
    assert torch.equal(y, x * 2.0)
    print(f"{scenario}: ok (rc {rcs})", flush=True)


if __name__ == "__main__":
    run(sys.argv[1])
