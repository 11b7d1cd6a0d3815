"""Host-side drop-in checks (no GPU): constructor limits fail at construction with a
documented message (P:66-83 accepts any value; the kernels cover input_dim 1..8 and 1..256
classes), the state-dict layout at non-default sizes, and per-replica dropout state under
DataParallel's replication (torch/nn/parallel/replicate.py shallow-copies __dict__)."""
import pytest

import pointnet_oracle as orc
from pcs_amd.model import PointNetSegmentation


@pytest.mark.parametrize("C,D", [(257, 4), (0, 4), (2, 9), (2, 0)])
def test_unsupported_sizes_raise_at_construction(C, D):
    with pytest.raises(ValueError, match="pcs_amd supports"):
        PointNetSegmentation(C, input_dim=D)


@pytest.mark.parametrize("C,D", [(20, 4), (3, 3), (64, 8), (65, 4), (256, 2)])
def test_state_dict_layout_generic_sizes(C, D):
    m = PointNetSegmentation(C, input_dim=D)
    sd = m.state_dict()
    assert list(sd.keys()) == orc.state_dict_keys(C, D)
    assert tuple(sd["conv1.weight"].shape) == (64, D, 1)
    assert tuple(sd["seg_conv4.weight"].shape) == (C, 128, 1)
    assert [n for n, _ in m.named_parameters()] == m._pnames


def test_replica_owns_dropout_state():
    m = PointNetSegmentation(2)
    r1 = m._replicate_for_data_parallel()
    r2 = m._replicate_for_data_parallel()
    assert r1._dstate is not m._dstate and r1._dstate is not r2._dstate
    assert r1._next_seed() != r2._next_seed()
    m2 = PointNetSegmentation(2)   # same base seed stream -> same replica seeds, in order
    q1 = m2._replicate_for_data_parallel()
    m2._replicate_for_data_parallel()
    r1b = PointNetSegmentation(2)._replicate_for_data_parallel()
    assert r1b._dstate.gen.initial_seed() == q1._dstate.gen.initial_seed()
