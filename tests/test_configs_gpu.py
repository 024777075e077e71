"""BASELINE.json configs 4 and 5 at full size (VERDICT r01 "next" #1, r02 #1).

Config 4 -- 8-camera array at 1080p D=128, gather + fuse, in both spellings:
SURVEY.md §8d's getCameraPairs(TO_CENTER_SMALL) = 12 <-> {6,7,8,11,13,16,17,18}
(/root/reference/src/functions.cpp:156-165), and BASELINE's own wording, a
2 x 4 grid with all 28 pairwise baselines (bench.py's grid8_all).  Each pair
is matched along its own baseline step, then the per-camera
median depth (§2.6).  Every map is bit-exact vs the threaded oracle
(oracle.sgm2), and every fused depth is bit-exact in f64 vs oracle.fuse_depth.

Config 5 -- 256 x 1080p D=192 pairs.  One pair bit-exact vs oracle.sgm, and
bench.py's batch route (consecutive pairs alternating over several
contexts/streams) byte-identical to the single-stream result for several
pairs.

Parity vs the reference itself is unpinned: the reference has
no SGM, no 2-D matcher and no fusion (its loop keeps the last pair,
CameraStereoVision.cpp:55).
"""
import numpy as np
import pytest
import torch

from stereovisionarray_amd import synth

pytestmark = [pytest.mark.gpu, pytest.mark.slow]

W, H = 1920, 1080
PITCH, F, PS = 0.05, 0.05, 0.036 / 1920      # CameraStereoVision.cpp:30-39
ORACLE_THREADS = 16                           # the GPU box's host budget
CENTER8 = [6, 7, 8, 11, 13, 16, 17, 18]       # TO_CENTER_SMALL partners of camera 12


def _grid():
    # the reference's 5x5 rig in grid units, camera 12 at (0, 0)
    return [(i % 5 - 2, i // 5 - 2) for i in range(25)]


@pytest.fixture(scope="module")
def center8_views():
    """The same synthetic scene bench.py's center8 workload uses."""
    D = 128
    g = _grid()
    kmax = max(synth.pair_step(g[12], g[j])[2] for j in CENTER8)
    dmax = min((D - 1) // kmax, 100)
    delta = synth.array_delta(H, W, dmax)
    cams = [12] + CENTER8
    views = dict(zip(cams, synth.array_views(H, W, [g[c] for c in cams], delta, seed=7)))
    return views, {}


@pytest.mark.parametrize("other", CENTER8)
def test_config4_center8_pair(ctx, sva, oracle, center8_views, other):
    views, maps = center8_views
    D = 128
    sx, sy, _ = synth.pair_step(_grid()[12], _grid()[other])
    p = sva.default_params(D=D, dmin=0, dir=sx, dir_y=sy)
    disp, _ = ctx.disparity_sgm(views[12], views[other], p)
    od, _ = oracle.sgm2(views[12], views[other], D, 0, sx, sy, subpixel=False,
                        threads=ORACLE_THREADS)
    assert np.array_equal(disp, od), f"pair 12->{other} step ({sx},{sy}): " \
        f"{int((disp != od).sum())} pixels differ"
    maps[other] = disp


def test_config4_center8_fusion(ctx, sva, oracle, center8_views):
    """8-map median depth around camera 12 (the gather + fuse step), bit-exact
    in f64; maps the per-pair tests did not leave behind are recomputed."""
    views, maps = center8_views
    g = _grid()
    stack, bases = [], []
    for j in CENTER8:
        sx, sy, k = synth.pair_step(g[12], g[j])
        if j not in maps:
            maps[j], _ = ctx.disparity_sgm(views[12], views[j],
                                           sva.default_params(D=128, dir=sx, dir_y=sy))
        stack.append(maps[j])
        bases.append(k * PITCH)
    stack = np.ascontiguousarray(np.stack(stack))
    depth, nv = ctx.fuse_depth(stack, bases, F, PS)
    exp, en = oracle.fuse_depth(stack, bases, F, PS)
    assert np.array_equal(nv, en)
    assert np.array_equal(depth.view(np.uint64), exp.view(np.uint64))
    assert (nv == 8).mean() > 0.5


# Config 4 in BASELINE's own wording (bench.py --workload grid8_all): an
# 8-camera array (2 x 4 grid), all 28 pairwise baselines at 1080p D=128, each
# matched along its reduced grid step.  The distinct steps are (-3,-1),
# (-2,-1), (-1,-1), (-1,0) at k = 1, 2, 3, (0,-1), (1,-1), (2,-1), (3,-1); every
# pair is compared with the threaded oracle, then the 7 per-camera median
# fusions (camera i fuses its pairs (i, j > i)) bit-exact in f64.
GRID8_PAIRS = synth.array_pairs(8)


@pytest.fixture(scope="module")
def grid8_views():
    D = 128
    g = synth.array_grid(2, 4)
    kmax = max(synth.pair_step(g[i], g[j])[2] for i, j in GRID8_PAIRS)
    dmax = min((D - 1) // kmax, 100)
    delta = synth.array_delta(H, W, dmax)
    views = synth.array_views(H, W, g, delta, seed=7)     # bench.py's grid8_all scene
    return g, views, {}


def test_grid8_all_steps_cover_the_verdict_list():
    g = synth.array_grid(2, 4)
    steps = {synth.pair_step(g[i], g[j]) for i, j in GRID8_PAIRS}
    assert {(sx, sy) for sx, sy, _ in steps} == {(-3, -1), (-2, -1), (-1, -1), (-1, 0), (0, -1),
                                                 (1, -1), (2, -1), (3, -1)}
    assert {k for sx, sy, k in steps if (sx, sy) == (-1, 0)} == {1, 2, 3}


@pytest.mark.parametrize("u", range(len(GRID8_PAIRS)))
def test_config4_grid8_all_pair(ctx, sva, oracle, grid8_views, u):
    g, views, maps = grid8_views
    i, j = GRID8_PAIRS[u]
    sx, sy, _ = synth.pair_step(g[i], g[j])
    p = sva.default_params(D=128, dmin=0, dir=sx, dir_y=sy)
    disp, _ = ctx.disparity_sgm(views[i], views[j], p)
    od, _ = oracle.sgm2(views[i], views[j], 128, 0, sx, sy, subpixel=False,
                        threads=ORACLE_THREADS)
    assert np.array_equal(disp, od), f"pair {i}->{j} step ({sx},{sy}): " \
        f"{int((disp != od).sum())} pixels differ"
    maps[u] = disp


def test_config4_grid8_all_fusion(ctx, sva, oracle, grid8_views):
    """The 7 fused maps of grid8_all (camera i over its pairs (i, j > i)),
    bit-exact in f64 vs oracle.fuse_depth; maps the per-pair tests did not
    leave behind are recomputed on the GPU."""
    g, views, maps = grid8_views
    n_groups = 0
    for i in range(7):
        stack, bases = [], []
        for u, (a, j) in enumerate(GRID8_PAIRS):
            if a != i:
                continue
            sx, sy, k = synth.pair_step(g[i], g[j])
            if u not in maps:
                maps[u], _ = ctx.disparity_sgm(views[i], views[j],
                                               sva.default_params(D=128, dir=sx, dir_y=sy))
            stack.append(maps[u])
            bases.append(k * PITCH)
        stack = np.ascontiguousarray(np.stack(stack))
        depth, nv = ctx.fuse_depth(stack, bases, F, PS)
        exp, en = oracle.fuse_depth(stack, bases, F, PS)
        assert np.array_equal(nv, en), f"camera {i}"
        assert np.array_equal(depth.view(np.uint64), exp.view(np.uint64)), f"camera {i}"
        assert (nv == len(bases)).mean() > 0.3, f"camera {i}"
        n_groups += 1
    assert n_groups == 7


def test_config5_pair_d192(ctx, sva, oracle):
    """One config-5 pair (seed 0) at 1920x1080 D=192,
    bit-exact vs the oracle; sub-pixel within 1e-5 px."""
    D = 192
    L, R, _ = synth.stereo_pair(H, W, D, 0, -1, seed=0)
    disp, sub = ctx.disparity_sgm(L, R, sva.default_params(D=D, subpixel=1))
    od, osub = oracle.sgm(L, R, D, 0, -1, subpixel=True, threads=ORACLE_THREADS)
    assert np.array_equal(disp, od)
    assert np.max(np.abs(sub - osub)) <= 1e-5


@pytest.mark.parametrize("n_ctx", [2, 3])
def test_config5_batch_route_streams(sva, oracle, torch_dev, n_ctx):
    """bench.py's config-5 route: pairs alternate over n_ctx contexts, each with
    its own HIP stream and workspaces (bench.py --streams); the maps must be
    byte-identical to the same pairs run one by one on one stream, and pair 0
    bit-exact vs the oracle (checked once, on the default route)."""
    D, n = 192, 6
    p = sva.default_params(D=D, dmin=0, dir=-1, subpixel=1)
    pairs = [synth.stereo_pair(H, W, D, 0, -1, seed=s)[:2] for s in range(n)]
    dl = [torch.from_numpy(a).to(torch_dev) for a, _ in pairs]
    dr = [torch.from_numpy(b).to(torch_dev) for _, b in pairs]
    ctxs, streams = [], []
    for _ in range(n_ctx):
        s = torch.cuda.Stream(torch_dev)
        c = sva.Context(torch_dev.index or 0)
        c.set_stream(s.cuda_stream)
        ctxs.append(c)
        streams.append(s)
    try:
        disp = torch.zeros((n, H, W), dtype=torch.int16, device=torch_dev)
        sub = torch.zeros((n, H, W), dtype=torch.float32, device=torch_dev)
        torch.cuda.synchronize()
        for j in range(n):
            ctxs[j % n_ctx].disparity_sgm_d(dl[j].data_ptr(), dr[j].data_ptr(), W, H, W, p,
                                        disp[j].data_ptr(), sub[j].data_ptr())
        for c in ctxs:
            c.synchronize()
        torch.cuda.synchronize()
        got = disp.cpu().numpy().view(np.uint16)
        gsub = sub.cpu().numpy()
        for j in range(n):                  # one stream, one pair at a time
            a, s1 = ctxs[0].disparity_sgm(pairs[j][0], pairs[j][1], p)
            assert np.array_equal(got[j], a), f"pair {j}"
            assert np.array_equal(gsub[j].view(np.uint32), s1.view(np.uint32)), f"pair {j}"
        if n_ctx == 2:
            od, _ = oracle.sgm(pairs[0][0], pairs[0][1], D, 0, -1, subpixel=False,
                               threads=ORACLE_THREADS)
            assert np.array_equal(got[0], od)
    finally:
        for c in ctxs:
            c.close()
