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


def test_batch_reuse_does_not_overwrite_maps_being_read(ctx, sva, torch_dev):
    """the caller reads batch 1's maps on the engine's device-0
    stream 0 while batch 2 is issued without a host sync.  Batch 2's local
    job on stream (0, 1) must not overwrite maps before that read has run
    (a spin kernel holds stream 0 back to open the window)."""
    if not hasattr(torch.cuda, "_sleep"):
        pytest.skip("torch.cuda._sleep not available")
    W, H, D, n = 200, 64, 64, 2
    m = sva.Multi([0], streams=2, flags=sva.SVA_MULTI_GATHER_RCCL)
    try:
        s0 = torch.cuda.Stream(torch_dev)
        m.context(0, 0).set_stream(s0.cuda_stream)    # the engine's stream (0, 0)
        pa = [synth.stereo_pair(H, W, D, 0, -1, seed=80 + i)[:2] for i in range(n)]
        pb = [synth.stereo_pair(H, W, D, 0, -1, seed=90 + i)[:2] for i in range(n)]
        p = sva.default_params(D=D)
        dev = [[torch.from_numpy(x).to(torch_dev) for x in q] for q in pa + pb]
        ja = [(dev[j][0].data_ptr(), dev[j][1].data_ptr(), p) for j in range(n)]
        jb = [(dev[n + j][0].data_ptr(), dev[n + j][1].data_ptr(), p) for j in range(n)]
        maps = torch.zeros((n, H, W), dtype=torch.int16, device=torch_dev)
        snap = torch.zeros_like(maps)
        torch.cuda.synchronize()
        m.batch_sgm_d(ja, W, H, W, maps.data_ptr())
        with torch.cuda.stream(s0):
            torch.cuda._sleep(200_000_000)              # ~0.1 s on stream (0, 0)
            snap.copy_(maps)                            # the caller's read of batch 1
        m.batch_sgm_d(jb, W, H, W, maps.data_ptr())
        m.synchronize()
        torch.cuda.synchronize()
        exp_a = np.stack([ctx.disparity_sgm(L, R, p)[0] for L, R in pa])
        exp_b = np.stack([ctx.disparity_sgm(L, R, p)[0] for L, R in pb])
        assert np.array_equal(snap.cpu().numpy().view(np.uint16), exp_a)
        assert np.array_equal(maps.cpu().numpy().view(np.uint16), exp_b)
    finally:
        m.close()


def test_batch_sub_planes_only_for_subpixel_jobs(ctx, sva, torch_dev):
    """with sub given, only jobs that set params.subpixel have
    their sub-pixel plane written (remote jobs included); the others keep the
    caller's contents instead of stale slot memory."""
    W, H, D, n = 150, 48, 64, 4
    m = sva.Multi([0], streams=2, flags=sva.SVA_MULTI_GATHER_RCCL | sva.SVA_MULTI_GATHER_ALL)
    try:
        pairs = [synth.stereo_pair(H, W, D, 0, -1, seed=70 + i)[:2] for i in range(n)]
        dl = [torch.from_numpy(a).to(torch_dev) for a, _ in pairs]
        dr = [torch.from_numpy(b).to(torch_dev) for _, b in pairs]
        ps = [sva.default_params(D=D, subpixel=j % 2) for j in range(n)]
        maps = torch.zeros((n, H, W), dtype=torch.int16, device=torch_dev)
        sub = torch.full((n, H, W), -3.0, dtype=torch.float32, device=torch_dev)
        torch.cuda.synchronize()
        for _ in range(2):                              # the second call reuses the slots
            m.batch_sgm_d([(dl[j].data_ptr(), dr[j].data_ptr(), ps[j]) for j in range(n)],
                          W, H, W, maps.data_ptr(), sub.data_ptr())
            m.synchronize()
        got = sub.cpu().numpy()
        for j, (L, R) in enumerate(pairs):
            if ps[j].subpixel:
                _, es = ctx.disparity_sgm(L, R, ps[j])
                assert np.array_equal(got[j].view(np.uint32), es.view(np.uint32)), j
            else:
                assert (got[j] == -3.0).all(), j
    finally:
        m.close()


def test_array_depth_rejects_mixed_invalid_in_group(sva):
    m = sva.Multi([0], streams=1, flags=sva.SVA_MULTI_GATHER_PEER)
    try:
        v = [np.zeros((24, 24), np.uint8)] * 3
        p0 = sva.default_params(D=64)
        p1 = sva.default_params(D=64)
        p1.invalid = 0
        jobs = [(0, 1, p0, 0.05), (0, 2, p1, 0.05)]
        with pytest.raises(sva.SvaError) as e:
            m.array_depth(v, jobs, [0, 2], 0.05, 1e-4)
        assert e.value.status == sva.SVA_ERR_INVALID_ARG
    finally:
        m.close()


def test_host_batch_repeated_calls_reuse_lanes(ctx, sva):
    """sva_batch_sgm keeps each context's pipeline lane between
    calls; repeated batches stay correct, and one context listed twice is
    refused (a context is not re-entrant)."""
    ctx2 = sva.Context(0)
    try:
        pairs = [synth.stereo_pair(70, 130, 64, 0, -1, seed=100 + i)[:2] for i in range(5)]
        p = sva.default_params(D=64, subpixel=1)
        first = sva.batch_sgm([ctx, ctx2], pairs, p)
        for _ in range(3):
            again = sva.batch_sgm([ctx, ctx2], pairs[::-1], p)
            for (d1, s1), (d2, s2) in zip(first[::-1], again):
                assert np.array_equal(d1, d2) and np.array_equal(s1, s2)
        with pytest.raises(sva.SvaError):
            sva.batch_sgm([ctx, ctx], pairs, p)
    finally:
        ctx2.close()


# ---- several devices: skipped on a one-GPU box ---------------------
def _devices(sva):
    n = min(sva.device_count(), 4)
    if n < 2:
        pytest.skip("needs >= 2 HIP devices")
    return list(range(n))


@pytest.mark.parametrize("mode", ["rccl", "peer"])
def test_batch_sgm_d_across_devices(ctx, sva, mode):
    """Remote jobs on devices[1..], one RCCL group over several communicators
    from one thread (or peer copies), per-device slots and gather events:
    every gathered map and sub-pixel map equals the single-context result."""
    devs = _devices(sva)
    W, H, D, n = 180, 72, 64, 2 * len(devs) + 1
    m = sva.Multi(devs, streams=2, flags=flags_of(sva, mode))
    try:
        pairs = [synth.stereo_pair(H, W, D, 0, -1, seed=120 + j)[:2] for j in range(n)]
        owner = [torch.device("cuda", devs[j % len(devs)]) for j in range(n)]
        dl = [torch.from_numpy(a).to(owner[j]) for j, (a, _) in enumerate(pairs)]
        dr = [torch.from_numpy(b).to(owner[j]) for j, (_, b) in enumerate(pairs)]
        p = sva.default_params(D=D, subpixel=1)
        d0 = torch.device("cuda", devs[0])
        maps = torch.zeros((n, H, W), dtype=torch.int16, device=d0)
        sub = torch.zeros((n, H, W), dtype=torch.float32, device=d0)
        for d in devs:
            torch.cuda.synchronize(d)
        for rep in range(2):
            order = list(range(n)) if rep == 0 else list(range(n))[::-1]
            m.batch_sgm_d([(dl[j].data_ptr(), dr[j].data_ptr(), p) for j in range(n)], W, H, W,
                          maps.data_ptr(), sub.data_ptr())
            m.synchronize()
            got = maps.cpu().numpy().view(np.uint16)
            gsub = sub.cpu().numpy()
            for j in order:
                ed, es = ctx.disparity_sgm(*pairs[j], p)
                assert np.array_equal(got[j], ed), (rep, j)
                assert np.array_equal(gsub[j].view(np.uint32), es.view(np.uint32)), (rep, j)
    finally:
        m.close()


@pytest.mark.parametrize("mode", ["rccl", "peer"])
def test_array_depth_across_devices(sva, oracle, mode):
    devs = _devices(sva)
    W, H, D = 160, 128, 64
    pitch_m, f, ps = 0.05, 0.05, 0.036 / 160
    grid, pairs, gs = _mini_rig()
    views = synth.array_views(H, W, grid, synth.array_delta(H, W, 14), seed=4)
    jobs, omaps = [], []
    for i, j in pairs:
        sx, sy, k = synth.pair_step(grid[i], grid[j])
        jobs.append((i, j, sva.default_params(D=D, dir=sx, dir_y=sy), k * pitch_m))
        omaps.append(oracle.sgm2(views[i], views[j], D, 0, sx, sy, subpixel=False)[0])
    m = sva.Multi(devs, streams=2, flags=flags_of(sva, mode))
    try:
        depth, nv, maps = m.array_depth(views, jobs, gs, f, ps, want_maps=True)
    finally:
        m.close()
    for j in range(len(pairs)):
        assert np.array_equal(maps[j], omaps[j]), pairs[j]
    for g in range(len(gs) - 1):
        sl = slice(gs[g], gs[g + 1])
        ez, en = oracle.fuse_depth(np.stack(omaps[sl]), [b for *_, b in jobs[sl]], f, ps)
        assert np.array_equal(nv[g], en)
        assert np.array_equal(depth[g].view(np.uint64), ez.view(np.uint64))
