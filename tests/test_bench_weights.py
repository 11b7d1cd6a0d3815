"""bench.py's multi-rank harness shares ONE class-weight vector (P:168-189, P:216): each rank's
label counts are summed over the process group, so every rank of a gloo world-2 run derives
bit-identical weights, equal to the reference formula over the concatenated batch; the single
process (world 1) keeps the local formula.  CPU only."""
import os
import sys

import numpy as np
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _rank_labels(rank, C):
    sys.path.insert(0, REPO)
    from pcs_amd.data import synthetic_batch
    _, lab, _ = synthetic_batch(1234 + rank, [4096, 3000], C, grid=16)
    return [lab[0], lab[1][:3000]]   # the scenes' own labels (the reference scans unpadded events)


def _worker(rank, world, port, C, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        sys.path.insert(0, REPO)
        import bench
        w = bench.shared_class_weights(_rank_labels(rank, C), C, world)
        q.put((rank, w))
    finally:
        dist.destroy_process_group()


def test_class_weights_identical_on_every_rank():
    sys.path.insert(0, REPO)
    from pcs_amd.data import class_weights
    C, world = 3, 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = 29700 + os.getpid() % 200
    ps = [ctx.Process(target=_worker, args=(r, world, port, C, q)) for r in range(world)]
    for p in ps:
        p.start()
    got = dict(q.get(timeout=240) for _ in range(world))
    for p in ps:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert got[0] == got[1]                                  # bitwise: one vector for the job
    concat = _rank_labels(0, C) + _rank_labels(1, C)
    ref = class_weights(concat, num_classes=C)
    np.testing.assert_allclose(got[0], ref, rtol=1e-12)
    own = class_weights(_rank_labels(0, C), num_classes=C)
    assert not np.allclose(own, ref, rtol=1e-6)              # the shards alone would differ


def test_class_weights_world_one_is_local():
    sys.path.insert(0, REPO)
    import bench
    from pcs_amd.data import class_weights
    labs = _rank_labels(0, 3)
    assert bench.shared_class_weights(labs, 3, 1) == class_weights(labs, num_classes=3)


def test_class_weights_skip_pads_even_when_they_dominate():
    """Pads (-1) never enter the weights: a scene padded far past its largest class gives the
    unpadded scene's weights (class_weights' Counter would take max_count from the pads)."""
    sys.path.insert(0, REPO)
    import bench
    from pcs_amd.data import class_weights
    own = _rank_labels(0, 3)
    padded = [np.concatenate([l, np.full(5 * l.size, -1, l.dtype)]) for l in own]
    assert bench.shared_class_weights(padded, 3, 1) == class_weights(own, num_classes=3)
    assert class_weights(padded, num_classes=3) != class_weights(own, num_classes=3)
