"""The C-ABI sharded RDM (vr_rdm_pearson_sharded, include/visreps_hip.h; SURVEY §8(b),(e)):
compute_rdm (visreps/analysis/rsa.py:59-93) over stimulus rows sharded across the ranks of
an RCCL communicator, for C callers without PyTorch.

CPU: the per-rank tile ranges (vr_rdm_sharded_range) partition the triangle, are cut only at
aligned boundaries (vr_rdm_range_aligned: bit-identical tiles to the one-GPU launch) and are
balanced. GPU: a one-rank communicator made through the library's own RCCL binding
(vr_rccl_unique_id / vr_rccl_comm_init) gives the split-Gram one-launch RDM bit for bit.
RCCL refuses two ranks on one device, so the multi-rank data path (padded row blocks, stats
unpack, per-rank tile ranges incl. empty ones, the packed-range exchange and the unpack of
other ranks' ranges, csrc/sharded.hip) runs through vr_rdm_pearson_sharded_comm with a
loopback all-gather: `world` host threads on one GPU, each a rank with its own stream,
workspace and output, the collective a barrier + device copies. Every rank's RDM must equal
the one-launch split-Gram RDM bit for bit."""
import ctypes

import numpy as np
import pytest

from visreps_amd._lib import VR_ALLGATHER_FN, VrComm, check, lib


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
    rc = L.vr_rdm_pearson_sharded(None, 5001, 10000, 64, 64, None, 10000, ctypes.c_float(1e-12), None, 0, 2,
                                  None, 0, None)
    assert rc != 0 and b"null comm" in L.vr_last_error()
    # more local rows than a block holds: refused before any collective runs
    calls = []
    comm = VrComm(2, 0, VR_ALLGATHER_FN(lambda *a: calls.append(a) or 0), None)
    rc = L.vr_rdm_pearson_sharded_comm(None, 5001, 10000, 64, 64, None, 10000, ctypes.c_float(1e-12),
                                       ctypes.byref(comm), None, 0, None)
    assert rc != 0 and b"local rows" in L.vr_last_error() and not calls
    rc = L.vr_rdm_pearson_sharded_comm(None, 0, 10000, 64, 64, None, 10000, ctypes.c_float(1e-12), None, None, 0, None)
    assert rc != 0 and b"null comm table" in L.vr_last_error()


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


def _hip_runtime():
    """The HIP runtime torch loaded (the library shares it), by its path in this process."""
    import os

    with open("/proc/self/maps") as f:
        paths = {ln.split()[-1] for ln in f if "libamdhip64" in ln}
    assert paths, "libamdhip64 not loaded"
    h = ctypes.CDLL(sorted(paths)[0], mode=os.RTLD_NOLOAD | os.RTLD_NOW)
    h.hipMemcpy.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int]
    h.hipStreamSynchronize.argtypes = [ctypes.c_void_p]
    return h


class _Loopback:
    """An in-process all-gather for `world` rank threads on one device (vr_comm.all_gather):
    each rank syncs its stream, publishes (send, recv), and after a barrier copies its send
    bytes into slot `rank` of every rank's recv; a second barrier ends the collective."""

    def __init__(self, world):
        import threading

        self.world, self.hip = world, _hip_runtime()
        self.barrier = threading.Barrier(world, timeout=120)
        self.slots = [None] * world
        self.calls = [0] * world
        self.fn = VR_ALLGATHER_FN(self._all_gather)  # one reference kept for the library's calls

    def _all_gather(self, send, recv, nbytes, user, stream):
        try:
            r = int(user) - 1
            assert self.hip.hipStreamSynchronize(stream) == 0
            self.slots[r] = (int(send), int(recv))
            self.barrier.wait()
            for j in range(self.world):
                dst = self.slots[j][1] + r * nbytes
                if dst != int(send):
                    assert self.hip.hipMemcpy(dst, send, nbytes, 3) == 0  # device to device
            assert self.hip.hipDeviceSynchronize() == 0
            self.calls[r] += 1
            self.barrier.wait()
            return 0
        except Exception:  # noqa: BLE001 -- a failed rank must release the others
            self.barrier.abort()
            return 1


@pytest.mark.gpu
@pytest.mark.parametrize("n,d,counts", [
    (3000, 4096, [1500, 1500]),
    (2990, 4096, [997, 996, 997]),                           # unequal, padded blocks
    (10000, 4096, [3334, 3333, 3333]),
    (9990, 2048, [1249, 1249, 1248, 1249, 1249, 1249, 1248, 1249]),
    (2990, 512, [374, 374, 373, 374, 374, 374, 373, 374]),   # world 8 with empty tile ranges
    (21, 64, [3, 3, 3, 0, 3, 3, 3, 3]),                      # a rank holding no rows
])
def test_sharded_multi_rank_loopback_equals_one_launch(dev, n, d, counts, monkeypatch):
    import threading

    import torch

    from visreps_amd.analysis import rsa as R

    L = lib()
    world = len(counts)
    assert sum(counts) == n and max(counts) <= -(-n // world)
    ranges = [_range(n, d, world, r) for r in range(world)]
    g = torch.Generator(device=dev).manual_seed(n + d + world)
    x = torch.relu(torch.randn(n, d, device=dev, generator=g))
    offs = np.concatenate([[0], np.cumsum(counts)])
    lb = _Loopback(world)
    comms = [VrComm(world, r, lb.fn, r + 1) for r in range(world)]
    wsb = int(L.vr_rdm_sharded_workspace(n, d, world))
    outs = [torch.full((n, n), float("nan"), device=dev) for _ in range(world)]
    wss = [torch.empty(wsb, dtype=torch.uint8, device=dev) for _ in range(world)]
    streams = [torch.cuda.Stream(device=dev) for _ in range(world)]
    torch.cuda.synchronize()
    rcs, errs = [None] * world, [None] * world

    def rank_main(r):
        torch.cuda.set_device(dev)
        xr = x[int(offs[r]):int(offs[r + 1])]
        rcs[r] = L.vr_rdm_pearson_sharded_comm(
            xr.data_ptr() if counts[r] else None, counts[r], n, d, d, outs[r].data_ptr(), n, ctypes.c_float(1e-12),
            ctypes.byref(comms[r]), wss[r].data_ptr(), wss[r].numel(), ctypes.c_void_p(streams[r].cuda_stream))
        if rcs[r] != 0:
            errs[r] = L.vr_last_error()
        else:
            streams[r].synchronize()

    th = [threading.Thread(target=rank_main, args=(r,)) for r in range(world)]
    for t in th:
        t.start()
    for t in th:
        t.join(timeout=300)
    assert not any(t.is_alive() for t in th), "a rank thread hung"
    assert rcs == [0] * world, errs
    assert lb.calls == [3] * world  # counts, plane blocks, packed tile ranges
    monkeypatch.setenv("VISREPS_GRAM", "split")  # the sharded path always runs the split Gram
    one = R.compute_rdm(x)
    for r in range(world):
        assert torch.equal(outs[r], one), (r, ranges)
    if n == 2990 and world == 8:
        assert any(b == a for a, b in ranges), ranges  # the case exercises an empty tile range
