import ctypes, os
import numpy as np
import torch
here = os.path.dirname(os.path.abspath(__file__))
lib = ctypes.CDLL(os.path.join(here, "libdbg.so"))
dev = "cuda"
g = (torch.arange(64 * 256) % 32768).to(torch.int16).view(64, 256).to(dev)
x = g.clone()
rc = torch.tensor([0, 0], dtype=torch.int32, device=dev)
slab = torch.zeros(65536, device=dev)
dump = torch.zeros(65536, dtype=torch.uint8, device=dev)
print("rc", lib.run_dbg(ctypes.c_void_p(g.data_ptr()), ctypes.c_void_p(x.data_ptr()), ctypes.c_long(64), ctypes.c_void_p(rc.data_ptr()), ctypes.c_void_p(slab.data_ptr()), ctypes.c_void_p(dump.data_ptr())))
d = dump.cpu().numpy()
fr = d[:64 * 32].view(np.int16).reshape(64, 16)
offs = d[16384:16384 + 256].view(np.int32)
for l in range(0, 64, 3):
    print(l, "off", offs[l], "f0", [(int(v) // 256, int(v) % 256) for v in fr[l, :8]])
