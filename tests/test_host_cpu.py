"""Host-side mirror of the reference trainer against golden vectors (no GPU needed)."""
import numpy as np
import pytest
import torch

from dcrecommend.optim.cyclic_scheduler import CyclicLRWithRestarts


@pytest.mark.parametrize("tag", ["a", "b"])
def test_scheduler_sequence(golden, tag):
    g = golden("scheduler.npz")
    B, n_train, period, t_mult, base_wd, epoch_size, nb = g[tag + "_cfg"]
    B, epoch_size, nb = int(B), int(epoch_size), int(nb)
    p = torch.nn.Parameter(torch.zeros(1))
    opt = torch.optim.Adam([p], 1e-3, (0.9, 0.99), 1e-8, float(base_wd))
    sch = CyclicLRWithRestarts(opt, B, epoch_size=epoch_size, restart_period=float(period),
                               t_mult=float(t_mult), policy="cosine")
    lrs, wds = [], []
    for _ in range(20):
        sch.step()
        for _ in range(nb):
            lrs.append(opt.param_groups[0]["lr"])
            wds.append(opt.param_groups[0]["weight_decay"])
            sch.batch_step()
    assert np.array_equal(np.array(lrs), g[tag + "_lr"])
    assert np.array_equal(np.array(wds), g[tag + "_wd"])
    sch.step()
    raised = 0
    try:
        for _ in range(nb + 5):
            sch.batch_step()
    except StopIteration:
        raised = 1
    assert raised == int(g[tag + "_raised"])


class _Len:
    def __init__(self, n):
        self.n = n

    def __len__(self):
        return self.n


@pytest.mark.parametrize("n,seed", [(95, 0), (100, 1), (1003, 2), (7, 3)])
def test_get_batches_matches_reference(golden, n, seed):
    """DCUEDataset.get_batches against the reference's own output (batches.npz): np.random.shuffle
    of the row order, chunks of ceil(len/k), the last chunk dropped when len % k != 0 -- including
    n = 7 with k = 10, where every chunk holds one row and the seventh is dropped
    (datasets/dcuedataset.py:189-201)."""
    from dcrecommend.datasets.dcuedataset import DCUEDataset
    g = golden("batches.npz")
    np.random.seed(seed)
    chunks = DCUEDataset.get_batches(_Len(n), k=10)
    assert np.array_equal(np.array([len(c) for c in chunks]), g["n%d_lens" % n])
    assert np.array_equal(np.array([x for c in chunks for x in c], dtype=np.int64), g["n%d_flat" % n])
