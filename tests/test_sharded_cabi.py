"""The C-ABI sharded RDM (vr_rdm_pearson_sharded, include/visreps_hip.h; SURVEY §8(b),(e)):
compute_rdm (visreps/analysis/rsa.py:59-93) over stimulus rows sharded across the ranks of
an RCCL communicator, for C callers without PyTorch.

CPU: the per-rank tile ranges (vr_rdm_sharded_range) partition the triangle, are cut only at
aligned boundaries (vr_rdm_range_aligned: bit-identical tiles to the one-GPU launch) and are
balanced. GPU: a one-rank communicator made through the library's own RCCL binding
(vr_rccl_unique_id / vr_rccl_comm_init) gives the split-Gram one-launch RDM bit for bit. More
ranks need more GPUs (RCCL refuses two ranks on one device): the multi-rank exchange runs
only on the driver's 8-GPU node."""
import ctypes

import numpy as np
import pytest

from visreps_amd._lib import check, lib


def _range(n, d, world, rank):
    a, b = ctypes.c_int64(), ctypes.c_int64()
    check(lib().vr_rdm_sharded_range(n, d, world, rank, ctypes.byref(a), ctypes.byref(b)), "vr_rdm_sharded_range")
    return a.value, b.value


@pytest.mark.parametrize("n,d", [(10000, 43264), (10000, 4096), (73000, 43264), (3000, 500), (300, 40)])
@pytest.mark.parametrize("world", [1, 2, 3, 8])
def test_sharded_ranges_partition_aligned_balanced(n, d, world):
    L = lib()
    total = int(L.vr_rdm_tile_count(n))
    ranges = [_range(n, d, world, r) for r in range(world)]
    assert ranges[0][0] == 0 and ranges[-1][1] == total
    for (a0, b0), (a1, b1) in zip(ranges[:-1], ranges[1:]):
        assert b0 == a1 and a0 <= b0
    for a, b in ranges:
        if b > a:
            assert L.vr_rdm_range_aligned(n, d, a, b) == 1, (n, d, world, a, b)
    if n >= 10000 and world <= 8:  # enough aligned boundaries for a balanced cut
        cost = np.array([L.vr_rdm_tile_cost(n, t) for t in range(total)], dtype=np.float64)
        load = [cost[a:b].sum() for a, b in ranges]
        assert max(load) <= 1.25 * cost.sum() / world, (n, d, world, load)


def test_sharded_workspace_and_argument_checks():
    L = lib()
    assert L.vr_rdm_sharded_workspace(10000, 4096, 8) > 0
    # more local rows than a block holds: refused before any RCCL call
    rc = L.vr_rdm_pearson_sharded(None, 5001, 10000, 64, 64, None, 10000, ctypes.c_float(1e-12), None, 0, 2,
                                  None, 0, None)
    assert rc != 0 and b"local rows" in L.vr_last_error()


@pytest.mark.gpu
@pytest.mark.parametrize("n,d", [(3000, 4096), (1000, 300)])
def test_sharded_one_rank_equals_one_launch(dev, n, d, monkeypatch):
    import torch

    from visreps_amd._lib import stream_of
    from visreps_amd.analysis import rsa as R

    L = lib()
    assert L.vr_rccl_available() == 1, "librccl.so.1 must be loadable on the GPU box"
    uid = (ctypes.c_char * 128)()
    check(L.vr_rccl_unique_id(uid), "vr_rccl_unique_id")
    comm = ctypes.c_void_p()
    check(L.vr_rccl_comm_init(ctypes.byref(comm), 1, uid, 0), "vr_rccl_comm_init")
    try:
        g = torch.Generator(device=dev).manual_seed(n + d)
        x = torch.relu(torch.randn(n, d, device=dev, generator=g))
        out = torch.full((n, n), float("nan"), device=dev)
        ws = torch.empty(int(L.vr_rdm_sharded_workspace(n, d, 1)), dtype=torch.uint8, device=dev)
        check(L.vr_rdm_pearson_sharded(x.data_ptr(), n, n, d, d, out.data_ptr(), n, ctypes.c_float(1e-12), comm, 0, 1,
                                       ws.data_ptr(), ws.numel(), stream_of(dev)), "vr_rdm_pearson_sharded")
        monkeypatch.setenv("VISREPS_GRAM", "split")  # the sharded path always runs the split Gram
        one = R.compute_rdm(x)
        assert torch.equal(out, one)
    finally:
        check(L.vr_rccl_comm_destroy(comm), "vr_rccl_comm_destroy")
