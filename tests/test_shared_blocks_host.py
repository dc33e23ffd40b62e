"""Host side of the shared packed input blocks (smt.ColumnBlockGroup): the union and its positions,
and the tile tables the wgrad kernel reads against them. No kernels run here."""
import torch

from sparse_matrix_tuning_amd.smt import smt


def test_group_union_positions_and_member_tables():
    q = smt.TileIndex([(15, 3), (0, 0)])
    k = smt.TileIndex([(1, 3), (2, 7)])
    v = smt.TileIndex([(0, 0), (3, 7), (1, 9)])
    grp = smt.ColumnBlockGroup({c for t in (q, k, v) for c in t.column_blocks()}, torch.device("cpu"))
    assert grp.col_blocks == [0, 3, 7, 9]
    assert grp.cb_dev.tolist() == [0, 3, 7, 9] and grp.cb_dev.dtype == torch.int32
    assert q.kernel_tiles(grp.pos) == [(15, 1), (0, 0)]
    assert k.kernel_tiles(grp.pos) == [(1, 1), (2, 2)]
    assert v.kernel_tiles(grp.pos) == [(0, 0), (3, 2), (1, 3)]
    # the member's own packing is unchanged beside it (first-use order of its own blocks)
    assert v.kernel_tiles(True) == [(0, 0), (3, 1), (1, 2)]
    assert v.kernel_tiles(False) == [(0, 0), (3, 7), (1, 9)]
    # a new map object (a re-selection) is not served from the cache of the old one
    other = {0: 3, 7: 0, 9: 1}
    assert v.kernel_tiles(other) == [(0, 3), (3, 0), (1, 1)]
    assert v.kernel_tiles(grp.pos) == [(0, 0), (3, 2), (1, 3)]
