"""Build a kernel-variant copy of libsmt_hip.so from the in-tree sources with extra -D flags, for
A/B timing in one GPU call (load it with SMT_HIP_LIB=<path>). Variants land in
scripts/diag/_variants/ (git-ignored; built .so files travel to the GPU box with the tree).

    python scripts/diag/build_variant.py ring2 -DSMT_DKV_RING=2
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from sparse_matrix_tuning_amd import build as b  # noqa: E402


def main(name, *defines):
    out_dir = os.path.join(os.path.dirname(os.path.abspath(__file__)), "_variants")
    os.makedirs(out_dir, exist_ok=True)
    out = os.path.join(out_dir, f"libsmt_hip_{name}.so")
    b.run_build(out, defines)
    print(out)


if __name__ == "__main__":
    main(*sys.argv[1:])
