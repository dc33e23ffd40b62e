"""Build the gfx950 HIP library ``_lib/libsmt_hip.so`` in-tree with hipcc.

The library is the only native product code: ``csrc/smt_kernels.hip`` (the SMT hot path, C ABI
``include/smt_hip.h``) and ``csrc/llama_kernels.hip`` (fused LLaMA elementwise ops, C ABI
``include/smt_model_ops.h``) and ``csrc/attn_kernels.hip`` (causal flash attention, C ABI
``include/smt_attention.h``) and ``csrc/fp8_kernels.hip`` (e4m3 quantisation of the fp8 path, C ABI
``include/smt_fp8.h``) compiled for ``--offload-arch=gfx950``. It is loaded with
ctypes by :mod:`sparse_matrix_tuning_amd._hip` (no torch types cross the boundary).
"""
from __future__ import annotations

import os
import shutil
import subprocess
import sys

PKG_DIR = os.path.dirname(os.path.abspath(__file__))
REPO_DIR = os.path.dirname(PKG_DIR)
SRCS = [os.path.join(PKG_DIR, "csrc", n) for n in ("smt_kernels.hip", "llama_kernels.hip", "attn_kernels.hip",
                                                   "fp8_kernels.hip")]
HEADERS = [os.path.join(REPO_DIR, "include", n) for n in ("smt_hip.h", "smt_model_ops.h", "smt_attention.h",
                                                          "smt_fp8.h")]
HEADERS += [os.path.join(PKG_DIR, "csrc", n) for n in ("silu_math.h", "fp8_math.h")]
LIB_DIR = os.path.join(PKG_DIR, "_lib")
LIB_PATH = os.path.join(LIB_DIR, "libsmt_hip.so")
ARCH = "gfx950"


def hipcc() -> str:
    for cand in (os.environ.get("HIPCC"), "/opt/rocm/bin/hipcc", shutil.which("hipcc")):
        if cand and os.path.exists(cand):
            return cand
    raise RuntimeError("hipcc not found (set HIPCC or install ROCm under /opt/rocm)")


def is_stale() -> bool:
    if not os.path.exists(LIB_PATH):
        return True
    t = os.path.getmtime(LIB_PATH)
    return any(os.path.getmtime(p) > t for p in (*SRCS, *HEADERS, __file__))


# Per-source extra flags. attn_kernels.hip: no SLP vectoriser (it paired adjacent scalar fp32 ops of
# the softmax into v_pk_* with pack/unpack moves around them; the kernels pack explicitly where it
# pays). At two waves per SIMD the lean kernels keep MFMA results in VGPRs by themselves; the
# one-wave-per-SIMD forward puts its O accumulators in AGPRs.
FILE_FLAGS = {"attn_kernels.hip": ["-fno-slp-vectorize"]}


def compile_commands(out: str, defines=()) -> list:
    """hipcc commands: one object per source (run in parallel), then the shared-library link."""
    base = [hipcc(), f"--offload-arch={ARCH}", "-O3", "-std=c++17", "-fPIC", "-Wall", "-Wno-unused-function",
            "-I", os.path.join(REPO_DIR, "include"), *defines]
    objs, cmds = [], []
    for src in SRCS:
        obj = out + "." + os.path.splitext(os.path.basename(src))[0] + ".o"
        objs.append(obj)
        cmds.append(base + FILE_FLAGS.get(os.path.basename(src), []) + ["-c", "-o", obj, src])
    link = [hipcc(), f"--offload-arch={ARCH}", "-shared", "-fPIC", "-o", out, *objs]
    return cmds, link, objs


def run_build(out: str, defines=(), verbose: bool = False) -> None:
    cmds, link, objs = compile_commands(out, defines)
    if verbose:
        for c in cmds + [link]:
            print(" ".join(c), file=sys.stderr)
    procs = [subprocess.Popen(c, stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True) for c in cmds]
    errs = []
    for c, p in zip(cmds, procs):
        so, se = p.communicate()
        if p.returncode != 0:
            errs.append(f"{' '.join(c)}\n{so}\n{se}")
    if not errs:
        res = subprocess.run(link, capture_output=True, text=True)
        if res.returncode != 0:
            errs.append(f"{' '.join(link)}\n{res.stdout}\n{res.stderr}")
    for o in objs:
        if os.path.exists(o):
            os.remove(o)
    if errs:
        raise RuntimeError("hipcc failed:\n" + "\n".join(errs))


def build(force: bool = False, verbose: bool = False) -> str:
    """Compile the HIP library if it is missing or older than its sources; return its path."""
    if not force and not is_stale():
        return LIB_PATH
    os.makedirs(LIB_DIR, exist_ok=True)
    # per-process scratch names: ranks of one node that find the library stale may build at once;
    # each renames its own complete result into place (atomic)
    tmp = f"{LIB_PATH}.tmp{os.getpid()}"
    run_build(tmp, verbose=verbose)
    os.replace(tmp, LIB_PATH)
    return LIB_PATH


if __name__ == "__main__":
    print(build(force="--force" in sys.argv, verbose=True))
