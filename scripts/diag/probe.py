import ctypes, os, sys
import numpy as np
import torch
here = os.path.dirname(os.path.abspath(__file__))
lib = ctypes.CDLL(os.path.join(here, "libprobe.so"))
tr = torch.zeros(256, dtype=torch.int16, device="cuda")
m0 = torch.zeros(1024, device="cuda"); m1 = torch.zeros(1024, device="cuda")
print("rc", lib.run_probes(ctypes.c_void_p(tr.data_ptr()), ctypes.c_void_p(m0.data_ptr()), ctypes.c_void_p(m1.data_ptr())))
t = tr.cpu().numpy().reshape(64, 4)
for l in range(0, 64, 1):
    vals = [(int(v) // 64, int(v) % 64) for v in t[l]]
    print("lane", l, "(row,col):", vals)
# mfma check
A = np.array([[(i * 16 + k) % 61 for k in range(16)] for i in range(32)], dtype=np.float64)
B0 = np.array([[1.0 if (k == (j % 16)) else 0.0 for j in range(32)] for k in range(16)])
B1 = np.array([[(k * 3 + j) % 7 for j in range(32)] for k in range(16)], dtype=np.float64)
D0 = m0.cpu().numpy().reshape(32, 32); D1 = m1.cpu().numpy().reshape(32, 32)
print("mfma mode0 ok:", np.array_equal(D0, A @ B0), " mode1 ok:", np.array_equal(D1, A @ B1))
if not np.array_equal(D1, A @ B1):
    print(D1[:4, :8]); print((A @ B1)[:4, :8])
