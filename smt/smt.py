"""``smt.smt`` of the reference (deepspeed/smt/smt.py) -> :mod:`sparse_matrix_tuning_amd.smt.smt`."""
from sparse_matrix_tuning_amd.smt.smt import (  # noqa: F401
    Block_dimension,
    LinearLayer_ChannelSparsity,
    LinearLayer_MatrixSparsity,
    SMTLinear,
    convert_linear_layer_to_channel_sparsity,
    convert_linear_layer_to_matrix_sparsity,
    convert_matrix_sparsity_to_linear_layer,
    freeze_unselected_channel_layer,
    freeze_unselected_matrix_layer,
    get_optimizer_qk_augment_grouped_parameters,
    get_optimizer_sparse_grouped_parameters,
    linearChannel,
    linearZ,
    recursive_getattr,
    recursive_setattr,
)
