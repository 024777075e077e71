"""The multi-GPU engine and the pipelined host batch on one MI355X
(VERDICT r01 "next" #4).

On the one-GPU box the engine runs one device with two streams; the gather is
exercised through a communicator of size 1 (RCCL self send/recv) or device-
local peer copies by routing device 0's own maps through the exchange
(SVA_MULTI_GATHER_ALL).  Every map must equal the single-context result and
the CPU oracle; the camera-array frame's fused depth is bit-exact in f64 vs
oracle.fuse_depth over oracle.sgm2 maps.
"""
import numpy as np
import pytest
import torch

from stereovisionarray_amd import synth

pytestmark = pytest.mark.gpu

MODES = ["rccl_all", "peer_all", "rccl", "peer"]


def flags_of(sva, mode):
    f = sva.SVA_MULTI_GATHER_PEER if mode.startswith("peer") else sva.SVA_MULTI_GATHER_RCCL
    return f | (sva.SVA_MULTI_GATHER_ALL if mode.endswith("_all") else 0)


@pytest.mark.parametrize("mode", MODES)
@pytest.mark.parametrize("D", [64, 128])
def test_batch_sgm_d(ctx, sva, oracle, torch_dev, mode, D):
    W, H, n = 210, 64, 5
    m = sva.Multi([0], streams=2, flags=flags_of(sva, mode))
    try:
        pairs = [synth.stereo_pair(H, W, D, 0, -1, seed=40 + i)[:2] for i in range(n)]
        dl = [torch.from_numpy(a).to(torch_dev) for a, _ in pairs]
        dr = [torch.from_numpy(b).to(torch_dev) for _, b in pairs]
        p = sva.default_params(D=D, subpixel=1)
        maps = torch.full((n, H, W), 7, dtype=torch.int16, device=torch_dev)
        sub = torch.zeros((n, H, W), dtype=torch.float32, device=torch_dev)
        torch.cuda.synchronize()
        m.batch_sgm_d([(dl[j].data_ptr(), dr[j].data_ptr(), p) for j in range(n)], W, H, W,
                      maps.data_ptr(), sub.data_ptr())
        m.synchronize()
        got = maps.cpu().numpy().view(np.uint16)
        gsub = sub.cpu().numpy()
        for j, (L, R) in enumerate(pairs):
            ed, es = ctx.disparity_sgm(L, R, p)
            assert np.array_equal(got[j], ed), f"pair {j}"
            assert np.array_equal(gsub[j].view(np.uint32), es.view(np.uint32)), f"pair {j}"
        od, _ = oracle.sgm(pairs[0][0], pairs[0][1], D, 0, -1, subpixel=False, threads=8)
        assert np.array_equal(got[0], od)
        # a second batch reuses the slots behind the first batch's gather
        m.batch_sgm_d([(dl[j].data_ptr(), dr[j].data_ptr(), p) for j in range(n)][::-1], W, H,
                      W, maps.data_ptr(), None)
        m.synchronize()
        again = maps.cpu().numpy().view(np.uint16)
        assert np.array_equal(again, got[::-1])
    finally:
        m.close()


def test_batch_sgm_d_mixed_steps_and_errors(ctx, sva, oracle, torch_dev):
    """Per-pair params (2-D array steps) and argument errors."""
    W, H, D = 96, 90, 64
    steps = [(0, -1), (-1, -1), (-1, 0), (1, 1)]
    m = sva.Multi([0], streams=2, flags=sva.SVA_MULTI_GATHER_RCCL | sva.SVA_MULTI_GATHER_ALL)
    try:
        imgs = [synth.stereo_pair2(H, W, D, 0, sx, sy, seed=5 + i)[:2]
                for i, (sx, sy) in enumerate(steps)]
        dl = [torch.from_numpy(a).to(torch_dev) for a, _ in imgs]
        dr = [torch.from_numpy(b).to(torch_dev) for _, b in imgs]
        ps = [sva.default_params(D=D, dir=sx, dir_y=sy) for sx, sy in steps]
        maps = torch.zeros((len(steps), H, W), dtype=torch.int16, device=torch_dev)
        torch.cuda.synchronize()
        m.batch_sgm_d([(dl[j].data_ptr(), dr[j].data_ptr(), ps[j]) for j in range(len(steps))],
                      W, H, W, maps.data_ptr())
        m.synchronize()
        got = maps.cpu().numpy().view(np.uint16)
        for j, (sx, sy) in enumerate(steps):
            od, _ = oracle.sgm2(imgs[j][0], imgs[j][1], D, 0, sx, sy, subpixel=False)
            assert np.array_equal(got[j], od), (sx, sy)
        with pytest.raises(sva.SvaError) as e:
            m.batch_sgm_d([(dl[0].data_ptr(), dr[0].data_ptr(), sva.default_params(D=300))], W, H,
                          W, maps.data_ptr())
        assert e.value.status == sva.SVA_ERR_INVALID_ARG
        # any D <= 256 runs padded to the next native width
        m.batch_sgm_d([(dl[2].data_ptr(), dr[2].data_ptr(), sva.default_params(D=50, dir=-1))],
                      W, H, W, maps.data_ptr())
        m.synchronize()
        od, _ = oracle.sgm2(imgs[2][0], imgs[2][1], 50, 0, -1, 0, subpixel=False)
        assert np.array_equal(maps[0].cpu().numpy().view(np.uint16), od)
        h = m.context_handle(0, 1)
        assert h
        with pytest.raises(sva.SvaError):
            m.context_handle(1, 0)
    finally:
        m.close()


def _mini_rig():
    """Camera 4 of a 3x3 grid against its 8 neighbours (a TO_CENTER_SMALL
    analogue), plus camera 0 against 1 and 3: two fusion groups."""
    grid = [(i % 3 - 1, i // 3 - 1) for i in range(9)]
    pairs = [(4, j) for j in (0, 1, 2, 3, 5, 6, 7, 8)] + [(0, 1), (0, 3)]
    return grid, pairs, [0, 8, 10]


@pytest.mark.parametrize("mode", ["rccl_all", "peer"])
def test_array_depth_matches_oracle(sva, oracle, mode):
    W, H, D = 160, 128, 64
    pitch_m, f, ps = 0.05, 0.05, 0.036 / 160
    grid, pairs, gs = _mini_rig()
    delta = synth.array_delta(H, W, 14)
    views = synth.array_views(H, W, grid, delta, seed=3)
    jobs, omaps = [], []
    for i, j in pairs:
        sx, sy, k = synth.pair_step(grid[i], grid[j])
        jobs.append((i, j, sva.default_params(D=D, dir=sx, dir_y=sy), k * pitch_m))
        od, _ = oracle.sgm2(views[i], views[j], D, 0, sx, sy, subpixel=False)
        omaps.append(od)
    m = sva.Multi([0], streams=2, flags=flags_of(sva, mode))
    try:
        depth, nv, maps = m.array_depth(views, jobs, gs, f, ps, want_maps=True)
        depth2, nv2, _ = m.array_depth(views, jobs, gs, f, ps)        # engine reuse
    finally:
        m.close()
    for j in range(len(pairs)):
        assert np.array_equal(maps[j], omaps[j]), pairs[j]
    for g in range(len(gs) - 1):
        sl = slice(gs[g], gs[g + 1])
        ez, en = oracle.fuse_depth(np.stack(omaps[sl]), [b for *_, b in jobs[sl]], f, ps)
        assert np.array_equal(nv[g], en)
        assert np.array_equal(depth[g].view(np.uint64), ez.view(np.uint64))
    assert np.array_equal(depth, depth2) and np.array_equal(nv, nv2)


def test_array_depth_rejects_bad_groups(sva):
    m = sva.Multi([0], streams=1, flags=sva.SVA_MULTI_GATHER_PEER)
    try:
        v = [np.zeros((20, 20), np.uint8)] * 2
        job = [(0, 1, sva.default_params(D=64), 0.05)]
        for gs in ([1, 1], [0, 2], [0, 0, 1]):
            with pytest.raises(sva.SvaError):
                m.array_depth(v, job, gs, 0.05, 1e-4)
    finally:
        m.close()


def test_host_batch_pipelined_with_failing_pair(ctx, sva):
    """sva_batch_sgm: per-context pipelines (pinned staging, copy streams); a
    bad pair reports its own status and the others still complete."""
    ctx2 = sva.Context(0)
    try:
        pairs = [synth.stereo_pair(80 + 4 * i, 150 - 2 * i, 64, 0, -1, seed=60 + i)[:2]
                 for i in range(7)]
        pairs[3] = (np.zeros((0, 0), np.uint8), np.zeros((0, 0), np.uint8))
        p = sva.default_params(D=64, subpixel=1)
        st = []
        outs = sva.batch_sgm([ctx, ctx2], pairs, p, statuses=st)
        assert st[3] == sva.SVA_ERR_INVALID_ARG
        assert all(s == sva.SVA_OK for i, s in enumerate(st) if i != 3)
        for i, ((L, R), (d, s)) in enumerate(zip(pairs, outs)):
            if i == 3:
                continue
            ed, es = ctx.disparity_sgm(L, R, p)
            assert np.array_equal(d, ed) and np.array_equal(s, es), i
    finally:
        ctx2.close()
