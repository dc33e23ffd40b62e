import ctypes, os
import torch
here = os.path.dirname(os.path.abspath(__file__))
lib = ctypes.CDLL(os.path.join(here, "libprobe.so"))
o0 = torch.zeros(256, dtype=torch.int16, device="cuda"); o1 = torch.zeros(256, dtype=torch.int16, device="cuda")
print("rc", lib.run_swz(ctypes.c_void_p(o0.data_ptr()), ctypes.c_void_p(o1.data_ptr())))
for name, o in (("plain", o0), ("swz", o1)):
    t = o.cpu().numpy().reshape(64, 4)
    bad = 0
    for l in range(64):
        gi = l >> 4; li = l & 15
        want = [((8 * (gi >> 1) + e) * 256 + 32 + 16 * (gi & 1) + li) for e in range(4)]
        if list(map(int, t[l])) != want:
            bad += 1
            if bad < 6: print(name, "lane", l, "got", [(int(v)//256, int(v)%256) for v in t[l]], "want", [(w//256, w%256) for w in want])
    print(name, "bad lanes", bad)
