import ctypes, os
import numpy as np
import torch
here = os.path.dirname(os.path.abspath(__file__))
lib = ctypes.CDLL(os.path.join(here, "libdbg.so"))
dev = "cuda"
g = (torch.arange(64 * 256) % 32768).to(torch.int16).view(64, 256).to(dev)
x = (torch.arange(64 * 256) % 32768).to(torch.int16).view(64, 256).to(dev) + 1
rc = torch.tensor([0, 0], dtype=torch.int32, device=dev)
slab = torch.zeros(65536, device=dev)
dump = torch.zeros(65536, dtype=torch.uint8, device=dev)
print("rc", lib.run_dbg(ctypes.c_void_p(g.data_ptr()), ctypes.c_void_p(x.data_ptr()), ctypes.c_long(64), ctypes.c_void_p(rc.data_ptr()), ctypes.c_void_p(slab.data_ptr()), ctypes.c_void_p(dump.data_ptr())))
d = dump.cpu().numpy().view(np.int16)
A = d[:16384]
bad = 0
for k in range(64):
    for f in range(256):
        off = k * 512 + ((2 * f) ^ ((k & 3) << 6))
        v = int(A[off // 2])
        if v != k * 256 + f:
            bad += 1
            if bad < 10: print("A k", k, "f", f, "got", (v // 256, v % 256))
print("bad A", bad)
