"""Time the register-resident RMSNorm kernels at the bench shape (T = 32768, hidden 4096) through the
C ABI: smt_rmsnorm_bwd_add (dy, x, dres read, dx written) and smt_add_rmsnorm_fwd (x, residual read,
h, y written); HIP events on the launch stream, HBM rate on the algorithmic bytes, and a checksum of
the outputs (variants must be bit-identical). Compare builds with SMT_HIP_LIB=<variant .so>."""
import hashlib
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from sparse_matrix_tuning_amd import _hip  # noqa: E402


def timeit(fn, iters=50):
    for _ in range(5):
        fn()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(iters):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / iters * 1e-3


def main():
    dev = torch.device("cuda", 0)
    T, H = 32768, 4096
    g = torch.Generator(device=dev).manual_seed(0)
    x = torch.randn(T, H, device=dev, generator=g).bfloat16()
    dy = torch.randn(T, H, device=dev, generator=g).bfloat16()
    dres = torch.randn(T, H, device=dev, generator=g).bfloat16()
    w = (1 + 0.1 * torch.randn(H, device=dev, generator=g)).bfloat16()
    rstd = torch.rand(T, device=dev, generator=g) + 0.5
    dx = torch.empty_like(x)
    h = torch.empty_like(x)
    y = torch.empty_like(x)
    rs = torch.empty(T, device=dev)
    lib = _hip.load()
    st = _hip._stream(dev)
    P = _hip._ptr

    def bwd():
        rc = lib.smt_rmsnorm_bwd_add(P(dy), H, P(x), H, P(w), P(rstd), P(dres), H, P(dx), H, T, H, 0, st)
        assert rc == 0

    def fwd():
        rc = lib.smt_add_rmsnorm_fwd(P(x), H, P(dres), H, P(w), P(h), H, P(y), H, P(rs), T, H, 1e-5, 0, st)
        assert rc == 0

    from sparse_matrix_tuning_amd import fused_llama as fl
    B, S, D = 16, 2048, 128
    qh = torch.randn(B, S, 32 * D, device=dev, generator=g).bfloat16().view(B, S, 32, D).transpose(1, 2)
    kh = torch.randn(B, S, 8 * D, device=dev, generator=g).bfloat16().view(B, S, 8, D).transpose(1, 2)
    cs = torch.randn(B, S, D, device=dev, generator=g).bfloat16()
    sn = torch.randn(B, S, D, device=dev, generator=g).bfloat16()
    rope_out = []

    def rope():
        rope_out[:] = fl._rope_launch("smt_rope_fwd", qh, kh, cs, sn)

    out = {"lib": os.path.basename(os.environ.get("SMT_HIP_LIB", "default")),
           "env": {k: v for k, v in os.environ.items() if k.startswith("SMT_ROPE")}}
    t = timeit(rope)
    hs = hashlib.sha256()
    for o in rope_out:
        hs.update(o.contiguous().view(torch.int16).cpu().numpy().tobytes())
    out["rope_fwd"] = {"us": round(t * 1e6, 1), "tb_s": round(2 * B * S * 40 * D * 2 / t / 1e12, 2),
                       "checksum": hs.hexdigest()[:12]}
    for name, fn, nbytes, outs in (("rmsnorm_bwd_add", bwd, 4 * T * H * 2, (dx,)),
                                   ("add_rmsnorm_fwd", fwd, 4 * T * H * 2, (h, y))):
        t = timeit(fn)
        hs = hashlib.sha256()
        for o in outs:
            hs.update(o.view(torch.int16).cpu().numpy().tobytes())
        out[name] = {"us": round(t * 1e6, 1), "tb_s": round(nbytes / t / 1e12, 2), "checksum": hs.hexdigest()[:12]}
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
