"""The HIP pieces of the multi-GPU RDM path (csrc/rdm.hip) on one GPU, emulating the
ranks of pipeline.gather_point_async / rdm_from_gathered in one process: shard-local
splits assembled into the gathered plane buffer must give, tile range by tile range, the
same entries as the one-process tile launch on the raw rows (bit for bit: identical plane
records and the same launch geometry), and the packed-range exchange must rebuild the
full RDM (with mirrors) exactly."""
import numpy as np
import pytest
import torch

from visreps_amd import pipeline as P
from visreps_amd.analysis import rsa as R
from visreps_amd.dataloaders.synthetic import shard_rows

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("n,d,world", [(700, 300, 2), (1500, 4096, 3), (3000, 2000, 8), (130, 33, 3)])
def test_planes_tiles_and_tile_exchange(dev, n, d, world, monkeypatch):
    monkeypatch.setenv("VISREPS_GRAM", "split")
    K = P.KERNELS
    g = torch.Generator(device=dev).manual_seed(n + d)
    x = torch.relu(torch.randn(n, d, device=dev, generator=g))
    # every rank's own split, gathered (here: concatenated in rank order) into plane rows
    parts = [K.split_rows(x[r.start:r.stop].contiguous(), 1e-12) for r in (shard_rows(n, q, world) for q in range(world))]
    planes = torch.zeros((K.plane_rows(n), K.plane_elems(d)), dtype=torch.int16, device=dev)
    planes[:n] = torch.cat([p[0] for p in parts])
    mean = torch.cat([p[1] for p in parts])
    std = torch.cat([p[2] for p in parts])
    ranges = P.tile_ranges(n, world)
    outs = []
    for t0, t1 in ranges:
        got = torch.full((n, n), float("nan"), device=dev)
        K.tiles_from_planes(planes, mean, std, n, d, got, t0, t1, 1e-12)
        ref = torch.full((n, n), float("nan"), device=dev)
        P.rdm_tiles_into(x, ref, t0, t1)
        assert torch.equal(torch.nan_to_num(got, nan=-7.0), torch.nan_to_num(ref, nan=-7.0))
        outs.append(got)
    # exchange: rank 0's matrix + every other range unpacked from its packed form
    full = outs[0].clone()
    for r, (t0, t1) in enumerate(ranges):
        packed = torch.empty((t1 - t0, P.TILE * P.TILE), device=dev)
        K.pack(outs[r], n, t0, t1, packed)
        if r:
            K.unpack(packed, n, t0, t1, full)
    assert not torch.isnan(full).any()
    assert torch.equal(full, full.T)
    one = R.compute_rdm(x)
    assert (full - one).abs().max().item() <= 2e-6  # per-range split-K order (pipeline.py doc)
