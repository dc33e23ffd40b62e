"""MI355X-native SMT (Sparse Matrix Tuning) block-sparse fine-tuning hot path.

Public surface mirrors the reference's ``smt.smt`` / ``smt.smt_helper`` modules
(``sparse_matrix_tuning_amd.smt.smt`` / ``.smt_helper``) plus a DeepSpeed-engine stand-in
(``sparse_matrix_tuning_amd.engine.initialize``). Compute goes through ``libsmt_hip.so``
(gfx950 HIP kernels behind the C ABI of ``include/smt_hip.h``).
"""
__version__ = "0.1.0"
