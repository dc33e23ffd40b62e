"""``smt.smt_helper`` of the reference (deepspeed/smt/smt_helper.py) ->
:mod:`sparse_matrix_tuning_amd.smt.smt_helper`."""
from sparse_matrix_tuning_amd.smt.smt_helper import (  # noqa: F401
    Block_dimension,
    L1_norm,
    L2_norm,
    abs_mean_,
    analyze_gradient_distribution,
    get_blocks,
    get_named_linears,
    mean_abs,
    select_channel_based_on_activation,
    select_submatrix_based_on_grads,
)
