"""Multi-process (world_size 2, gloo, CPU) tests of the shard/gather logic
used by bench.py --gpus N: unit i -> rank i mod N, one gather
of the disparity maps to rank 0, byte-identical to the single-rank result."""
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from stereovisionarray_amd import dist as sdist


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def fake_map(u, H=6, W=10):
    """Deterministic per-unit 'disparity map' (stands in for the GPU output)."""
    g = torch.Generator().manual_seed(1000 + u)
    return torch.randint(0, 65535, (H, W), generator=g, dtype=torch.int32).to(torch.int16)


def _worker(rank, world, port, n_units, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        mine = sdist.shard(n_units, rank, world)
        local = torch.stack([fake_map(u) for u in mine]) if mine else torch.zeros((0, 6, 10),
                                                                                  dtype=torch.int16)
        out = sdist.gather_maps(local, n_units)
        chk, ok = sdist.gather_maps_checked(local, n_units)
        if rank == 0:
            exp = torch.stack([fake_map(u) for u in range(n_units)])
            q.put(("ok", bool(torch.equal(out, exp)) and bool(torch.equal(chk, exp)) and ok))
        else:
            q.put(("ok", out is None and chk is None and ok))
    except Exception as e:  # pragma: no cover - surfaced through the queue
        q.put(("err", repr(e)))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,n_units", [(2, 8), (2, 5), (2, 1), (3, 7)])
def test_gather_matches_single_rank(world, n_units):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, n_units, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=120) for _ in procs]
    for p in procs:
        p.join(timeout=60)
    assert all(r == ("ok", True) for r in res), res


def test_checksums_detect_swaps_and_byte_errors():
    maps = torch.stack([fake_map(u) for u in range(4)])
    base = sdist.checksums(maps)
    assert len(set(base.tolist())) == 4
    swapped = maps[[1, 0, 2, 3]]
    assert not torch.equal(sdist.checksums(swapped), base)
    flipped = maps.clone()
    flipped[2, 3, 4] ^= 1
    got = sdist.checksums(flipped)
    assert got[2] != base[2] and torch.equal(got[[0, 1, 3]], base[[0, 1, 3]])
    rolled = torch.roll(maps, 1, dims=2)          # a shifted row layout
    assert not torch.equal(sdist.checksums(rolled), base)


def test_shard_covers_every_unit_once():
    for world in (1, 2, 4, 8):
        for n in (0, 1, 7, 8, 256):
            seen = sorted(u for r in range(world) for u in sdist.shard(n, r, world))
            assert seen == list(range(n))
            assert max((len(sdist.shard(n, r, world)) for r in range(world)), default=0) \
                <= sdist.slots(n, world)
