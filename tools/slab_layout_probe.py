"""Driver of tools/slab_layout_probe.hip (build: hipcc --offload-arch=gfx950 -O3 -shared -fPIC
tools/slab_layout_probe.hip -o tools/slab_layout_probe.so): device time of the slab fill and of the fixed-order
reduce for the workgroup-major and chunk-major layouts, HIP events over 20 launches after 5 warm-up launches,
three alternations; the two reduces' outputs must be bit-identical."""
import ctypes
import os

import torch

here = os.path.dirname(os.path.abspath(__file__))
lib = ctypes.CDLL(os.path.join(here, "slab_layout_probe.so"))
S = 32 * 2560
slab = torch.empty(256 * S, device="cuda")
outs = [torch.empty(S, device="cuda") for _ in range(2)]
st = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)


def timed(layout, what, n=20):
    for _ in range(5):
        assert lib.probe_slab(layout, what, ctypes.c_void_p(slab.data_ptr()), ctypes.c_longlong(S),
                              ctypes.c_void_p(outs[layout].data_ptr()), st) == 0
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(n):
        lib.probe_slab(layout, what, ctypes.c_void_p(slab.data_ptr()), ctypes.c_longlong(S),
                       ctypes.c_void_p(outs[layout].data_ptr()), st)
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) * 1e3 / n


def fill_then_reduce(layout, n=20):
    """The step's order: fill (the backward) then reduce, timed as the pair, and the reduce alone behind a fill."""
    tot = 0.0
    for _ in range(n):
        lib.probe_slab(layout, 0, ctypes.c_void_p(slab.data_ptr()), ctypes.c_longlong(S), None, st)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        lib.probe_slab(layout, 1, ctypes.c_void_p(slab.data_ptr()), ctypes.c_longlong(S),
                       ctypes.c_void_p(outs[layout].data_ptr()), st)
        e1.record()
        torch.cuda.synchronize()
        tot += e0.elapsed_time(e1) * 1e3
    return tot / n


mb = 256 * S * 4 / 1e6
for rep in range(3):
    for layout in (0, 1):
        f = timed(layout, 0)
        r = timed(layout, 1)
        rr = fill_then_reduce(layout)
        print(f"layout {layout} ({'wg-major' if layout == 0 else 'chunk-major'}): fill {f:7.2f} us "
              f"({mb / f:5.2f} TB/s)  reduce back-to-back {r:7.2f} us ({mb / r:5.2f} TB/s)  "
              f"reduce behind a fill {rr:7.2f} us ({mb / rr:5.2f} TB/s)", flush=True)
print("outputs bit-identical:", torch.equal(outs[0], outs[1]))
