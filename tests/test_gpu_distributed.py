"""The HIP pieces of the multi-GPU RDM path (csrc/rdm.hip) on one GPU, emulating the ranks
of pipeline.ShardedRDMs in one process.

* Aligned pieces (vr_rdm_range_aligned: cut at the wide kernel's super-tile rows, the
  remainder rows with the last piece) computed separately, packed and unpacked into one
  matrix, rebuild the one-launch RDM bit for bit -- at D >= 4096, where the one-launch RDM
  runs the wide kernel and split-K: every tile is summed in the same order whatever piece
  holds it, so RDMs (and the exact-integer scores) do not depend on the world size.
* The schedule's cuts are aligned for every world size at the bench's N.
* Unaligned ranges (the legacy tile-range API) still assemble within fp32 rounding.
* The pre-split plane entry points (vr_rdm_split_rows_f32 + vr_rdm_pearson_tiles_planes)
  equal the one-launch tiles on the raw rows.
"""
import ctypes

import numpy as np
import pytest
import torch

from visreps_amd import pipeline as P
from visreps_amd._lib import check, lib, stream_of, workspace
from visreps_amd.analysis import rsa as R
from visreps_amd.dataloaders.synthetic import shard_rows

pytestmark = pytest.mark.gpu


def _assemble(x, n, cuts):
    """Pieces [cuts[i], cuts[i+1]) computed into separate matrices, exchanged packed."""
    K = P.KERNELS
    full = None
    for a, b in zip(cuts[:-1], cuts[1:]):
        part = torch.full((n, n), float("nan"), device=x.device)
        K.tiles_from_rows(x, part, a, b, 1e-12)
        packed = torch.empty((b - a, P.TILE * P.TILE), device=x.device)
        K.pack(part, n, a, b, packed)
        if full is None:
            full = part
        else:
            K.unpack(packed, n, a, b, full)
            del part
    return full


@pytest.mark.parametrize("n,d,pieces", [(10000, 4096, 2), (10000, 4096, 5), (6000, 43264, 3), (7300, 9000, 8)])
def test_aligned_pieces_bit_identical_to_one_launch(dev, n, d, pieces):
    g = torch.Generator(device=dev).manual_seed(n + d)
    x = torch.relu(torch.randn(n, d, device=dev, generator=g))
    assert int(lib().vr_rdm_wide_rows(n, d)) > 0  # the one-launch RDM uses the wide kernel
    bnd = P.aligned_boundaries(n, d)
    assert len(bnd) > pieces
    cum = P._tile_cum_cost(n)
    cuts = sorted({0, len(cum) - 1} | {min(bnd, key=lambda t: abs(cum[t] - cum[-1] * j / pieces))
                                        for j in range(1, pieces)})
    for a, b in zip(cuts[:-1], cuts[1:]):
        assert lib().vr_rdm_range_aligned(n, d, a, b) == 1
    one = R.compute_rdm(x)
    got = _assemble(x, n, cuts)
    assert torch.equal(got, one)


@pytest.mark.parametrize("world", [2, 3, 4, 8])
def test_schedule_pieces_are_aligned_at_bench_size(dev, world):
    from bench import LAYERS  # noqa: F401  (bench.py's point list)
    dims = {"conv1_pre": 290400, "conv1_post": 290400, "conv2_pre": 186624, "conv2_post": 186624,
            "conv3_pre": 64896, "conv3_post": 64896, "conv4_pre": 64896, "conv4_post": 64896,
            "conv5_pre": 43264, "conv5_post": 43264, "fc1_pre": 4096, "fc1_post": 4096,
            "fc2_pre": 4096, "fc2_post": 4096}
    rois = {"V1": 2000, "V2": 2000, "V3": 2000, "hV4": 1000}
    s = P.make_schedule(10000, dims, list(dims), rois, world)
    width = dict(dims)
    for (kind, name), pcs in s.pieces.items():
        d = width[name] if kind == "m" else rois[name]
        for pc in pcs:
            assert lib().vr_rdm_range_aligned(10000, d, pc.t0, pc.t1) == 1, (name, pc)


@pytest.mark.parametrize("world", [3, 8])
def test_unaligned_ranges_match_within_rounding(dev, world):
    n, d = 3000, 4096
    g = torch.Generator(device=dev).manual_seed(world)
    x = torch.relu(torch.randn(n, d, device=dev, generator=g))
    full = R.compute_rdm(x)
    got = _assemble(x, n, [a for a, _ in P.tile_ranges(n, world)] + [int(lib().vr_rdm_tile_count(n))])
    assert torch.equal(got, got.T)
    assert (got - full).abs().max().item() <= 2e-6


@pytest.mark.parametrize("n,d,world", [(700, 300, 2), (1500, 4096, 3), (130, 33, 3)])
def test_presplit_planes_equal_row_tiles(dev, n, d, world, monkeypatch):
    monkeypatch.setenv("VISREPS_GRAM", "split")
    L = lib()
    g = torch.Generator(device=dev).manual_seed(n + d)
    x = torch.relu(torch.randn(n, d, device=dev, generator=g))
    prow, pel = int(L.vr_rdm_plane_rows(n)), int(L.vr_rdm_plane_row_bytes(d)) // 2
    planes = torch.zeros((prow, pel), dtype=torch.int16, device=dev)
    mean = torch.empty(n, device=dev)
    std = torch.empty(n, device=dev)
    for q in range(world):  # every rank splits its own rows
        r = shard_rows(n, q, world)
        xs = x[r.start:r.stop].contiguous()
        check(L.vr_rdm_split_rows_f32(xs.data_ptr(), xs.size(0), d, d, ctypes.c_float(1e-12),
                                      mean[r.start:].data_ptr(), std[r.start:].data_ptr(),
                                      planes[r.start:].data_ptr(), stream_of(dev)), "split")
    for t0, t1 in P.tile_ranges(n, world):
        got = torch.full((n, n), float("nan"), device=dev)
        ws = workspace.get(dev, L.vr_rdm_planes_tiles_workspace(n, d, t0, t1), "rdm")
        check(L.vr_rdm_pearson_tiles_planes(planes.data_ptr(), mean.data_ptr(), std.data_ptr(), n, d,
                                            got.data_ptr(), n, ctypes.c_float(1e-12), t0, t1, ws.data_ptr(),
                                            ws.numel(), stream_of(dev)), "tiles_planes")
        ref = torch.full((n, n), float("nan"), device=dev)
        P.rdm_tiles_into(x, ref, t0, t1)
        assert torch.equal(torch.nan_to_num(got, nan=-7.0), torch.nan_to_num(ref, nan=-7.0))
    assert np.isfinite(std.cpu().numpy()).all()


def test_bench_extract_split_equals_fp32_path(dev, monkeypatch):
    """bench.extract_split (the Gram prepass fused into extraction): the RDMs from its split
    rows equal the RDMs of bench.extract's fp32 feature buffers bit for bit, and the kept
    phase-1 rows equal the fp32 rows."""
    import os

    monkeypatch.setenv("VISREPS_GRAM", "split")
    # bench.py turns on cudnn.benchmark and MIOpen's find mode at import; the two extractions
    # below must run the same convolution algorithms (as tests/test_benchsize.py's fixture)
    prev = torch.backends.cudnn.benchmark, os.environ.get("MIOPEN_FIND_MODE")
    import bench
    torch.backends.cudnn.benchmark = prev[0]
    if prev[1] is None:
        os.environ.pop("MIOPEN_FIND_MODE", None)
    else:
        os.environ["MIOPEN_FIND_MODE"] = prev[1]
    from visreps_amd.dataloaders.synthetic import make_images
    from visreps_amd.models.custom_model import CustomCNN
    from visreps_amd.models.utils import FeatureExtractor

    torch.manual_seed(0)
    model = CustomCNN(num_classes=1000).to(dev).eval()
    ex = FeatureExtractor(model, ["conv5", "fc1"], extract_pre_and_post=True)
    n = 300
    images = make_images(range(n), device=dev)
    keep = np.array([3, 77, 150, 299, 0])
    full = bench.extract(ex, images, 64)
    split, sel = bench.extract_split(ex, images, 64, keep)
    total = int(lib().vr_rdm_tile_count(n))
    for p, x in full.items():
        assert torch.equal(sel[p], x[torch.as_tensor(keep, device=dev)])
        one = torch.empty((n, n), device=dev)
        P.rdm_tiles_into(x, one, 0, total)
        got = torch.empty((n, n), device=dev)
        P.KERNELS.tiles_from_planes(split[p], n, got, 0, total, 1e-12)
        assert torch.equal(got, one), p


def _gloo_rdm_worker(rank, world, port, n, d, out_dir):
    import os

    import torch.distributed as dist

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    torch.cuda.set_device(0)
    dev = torch.device("cuda", 0)
    g = torch.Generator(device=dev).manual_seed(30000)
    x = torch.relu(torch.randn(n, d, device=dev, generator=g))  # the same rows on every rank
    rows = shard_rows(n, rank, world)
    x_local = x[rows.start:rows.stop].clone()
    if rank != 0:
        del x
    torch.cuda.empty_cache()
    got = P.distributed_rdm(x_local, n, dist.group.WORLD)
    del x_local
    if rank == 0:
        one = torch.empty((n, n), dtype=torch.float32, device=dev)
        P.KERNELS.tiles_from_rows(x, one, 0, int(lib().vr_rdm_tile_count(n)), 1e-12)
        equal = bool(torch.equal(got, one))
        with open(os.path.join(out_dir, "equal.txt"), "w") as f:
            f.write(f"{int(equal)} {n} {d}\n")
    dist.barrier()
    dist.destroy_process_group()


def test_gloo_distributed_rdm_30k_on_one_gpu(dev, tmp_path):
    """distributed_rdm (pipeline.ShardedRDMs: row exchange to the owners, aligned
    pieces, packed piece exchange) at world 2 -- both ranks on this GPU over gloo, the
    orchestration RCCL runs on the 8-GPU node -- at 30,000 x 43,264 (5.2 GB of rows, 3.6 GB
    RDM): torch.equal with the one-launch RDM."""
    import socket

    import torch.multiprocessing as mp

    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    n, d = 30000, 43264
    mp.spawn(_gloo_rdm_worker, args=(2, port, n, d, str(tmp_path)), nprocs=2, join=True)
    flag, n_, d_ = open(tmp_path / "equal.txt").read().split()
    assert flag == "1" and int(n_) == n and int(d_) == d
