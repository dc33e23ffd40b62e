import os, sys
import torch
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from sparse_matrix_tuning_amd import _hip
dev = torch.device("cuda")
rc = _hip.tile_table([(0, 0)], dev)
for (t, a, b) in [(0, 0, 0), (0, 1, 0), (0, 0, 1), (0, 5, 9), (1, 0, 0), (3, 0, 0), (4, 0, 0), (8, 0, 0), (16, 0, 0), (17, 33, 70), (63, 200, 130), (0, 31, 0), (0, 32, 0), (0, 0, 32), (0, 130, 0), (0, 0, 65)]:
    g = torch.zeros(64, 256); x = torch.zeros(64, 256)
    g[t, a] = 1.0; x[t, b] = 1.0
    out = torch.empty(256, 256, device=dev)
    _hip.tile_wgrad(g.bfloat16().to(dev), x.bfloat16().to(dev), rc, out)
    o = out.cpu()
    nz = (o != 0).nonzero().tolist()
    print(f"t={t} m={a} n={b} -> nonzeros {nz[:6]} (count {len(nz)}) vals {[o[i][j].item() for i,j in nz[:3]]}")
# dense random small check: which fraction matches
g = torch.randn(64, 256).bfloat16(); x = torch.randn(64, 256).bfloat16()
out = torch.empty(256, 256, device=dev)
_hip.tile_wgrad(g.to(dev), x.to(dev), rc, out)
truth = g.double().t() @ x.double()
d = (out.cpu().double() - truth).abs()
print("max err", d.max().item(), "frac ok", (d < 1e-3).float().mean().item())
