"""Measure the v_mfma_scale_f32_32x32x64_f8f6f4 (e4m3 x e4m3) lane maps that wgrad_mx_kernel relies
on, with one-hot operands (the evidence behind mx_frag in csrc/smt_kernels.hip; result committed as
profiles/r02_mx_probe.json). Build first, on the CPU side:
    hipcc --offload-arch=gfx950 -O2 -shared -fPIC scripts/mx_probe.hip -o scripts/_probe/libmxprobe.so
Findings: A/B byte j of lane (r, h) pair at the same k (rows / cols = lane & 31, standard 32x32 C
map); the lane's scale (opsel 0: byte 0) covers 32 k of its row; the k of byte j is 16h + j for
j < 16 and 32 + 16h + (j - 16) otherwise, so k-block h = {bytes 0-15 of both halves' lanes ...}:
exactly, the lane-h scale multiplies bytes 16h.. of k-block h (experiment 4)."""
import ctypes, json, os, sys
import torch

lib = ctypes.CDLL(os.path.join(os.path.dirname(__file__), "_probe", "libmxprobe.so"))
ONE = 0x38                                                  # e4m3 1.0


def run(a, b, sa, sb):
    W = a.shape[0]
    d = torch.zeros(W, 64, 16, device="cuda")
    rc = lib.run_probe(*[ctypes.c_void_p(t.data_ptr()) for t in (a, b, sa, sb, d)], W)
    assert rc == 0, rc
    return d.cpu()


def cmap(d):
    """[W, 64, 16] accumulators -> [W, 32 rows, 32 cols] with the documented 32x32 C map."""
    out = torch.zeros(d.shape[0], 32, 32)
    for l in range(64):
        for i in range(16):
            out[:, (i & 3) + 8 * (i >> 2) + 4 * (l >> 5), l & 31] = d[:, l, i]
    return out


def as_words(bytes_):                                     # [W, 64, 32] uint8 -> int32 [W, 64, 8]
    return bytes_.contiguous().view(torch.int32).cuda()


res = {}
# experiment 1: A one-hot at (L, j); B byte (l, j') = e4m3 code 1 + 32*(l>>5) + j' (exact small values)
W = 64 * 32
a = torch.zeros(W, 64, 32, dtype=torch.uint8)
for w in range(W):
    a[w, w // 32, w % 32] = ONE
codes = torch.tensor([[1 + 32 * (l >> 5) + j for j in range(32)] for l in range(64)], dtype=torch.uint8)
b = codes.expand(W, 64, 32).clone()
vals = codes.view(torch.float8_e4m3fn).float()
s127 = torch.full((W, 64), 127, dtype=torch.int32).cuda()
D = cmap(run(as_words(a), as_words(b), s127, s127))
amap = {}
for w in range(W):
    L, j = w // 32, w % 32
    nz = (D[w] != 0).nonzero().tolist()
    rows = sorted({r for r, _ in nz})
    pair = {}
    for r, n in nz:
        v = D[w, r, n].item()
        hit = ((vals - v).abs() < 1e-9).nonzero().tolist()
        pair[n] = hit
    amap[f"{L},{j}"] = {"rows": rows, "pairs": {str(k): v for k, v in list(pair.items())[:4]}}
res["A_onehot"] = amap
# experiment 2: all ones, A scale 128 on one lane L -> which (row, k) the lane's scale covers
W2 = 64
a2 = torch.full((W2, 64, 32), ONE, dtype=torch.uint8)
sa = torch.full((W2, 64), 127, dtype=torch.int32)
for w in range(W2):
    sa[w, w] = 128
D2 = cmap(run(as_words(a2), as_words(a2.clone()), sa.cuda(), torch.full((W2, 64), 127, dtype=torch.int32).cuda()))
res["A_scale"] = {str(w): {"rows": sorted({r for r, _ in (D2[w] != 64).nonzero().tolist()}),
                          "value": sorted({D2[w, r, c].item() for r, c in (D2[w] != 64).nonzero().tolist()})}
                  for w in range(W2)}
# experiment 3: scale byte position (opsel 0): scale word 0x7f7f7f80 / 0x807f7f7f on lane 0
sa3 = torch.full((2, 64), 127, dtype=torch.int32)
sa3[0, 0] = 0x7F7F7F80
sa3[1, 0] = int(0x807F7F7F - (1 << 32))
D3 = cmap(run(as_words(a2[:2]), as_words(a2[:2].clone()), sa3.cuda(), torch.full((2, 64), 127, dtype=torch.int32).cuda()))
res["opsel0_low_byte"] = [sorted({D3[w, r, c].item() for r, c in (D3[w] != 64).nonzero().tolist()}) for w in range(2)]
# experiment 4: which A bytes does the scale of B lane 32 (h = 1) multiply? A one-hot at (lane 0 or 32,
# byte j), B all ones, B scale of lane 32 = 2.0: D[0][0] = 2 exactly for the bytes in k-block 1
sb4 = torch.where(torch.arange(64) == 32, 128, 127).int().expand(32, 64).contiguous().cuda()
for L in (0, 32):
    a4 = torch.zeros(32, 64, 32, dtype=torch.uint8)
    for j in range(32):
        a4[j, L, j] = ONE
    D4 = cmap(run(as_words(a4), as_words(a2[:32].clone()), s127[:32], sb4))
    res[f"kblock1_bytes_of_lane{L}"] = [j for j in range(32) if D4[j, 0, 0].item() == 2.0]
json.dump(res, open(sys.argv[1], "w"))
print("ok", res["A_scale"]["0"], res["A_scale"]["32"], res["opsel0_low_byte"], res["kblock1_bytes_of_lane0"],
      res["kblock1_bytes_of_lane32"])
