"""Multi-GPU engine host logic without a device: the shard
plan that sva_batch_sgm_d / sva_array_depth follow (pair j -> device j mod N,
round-robin over the device's contexts, consecutive slots per context), and
argument checks that fail before any device is touched."""
import numpy as np
import pytest

import stereovisionarray_amd as sva


@pytest.mark.parametrize("nd,spd,n", [(1, 1, 1), (1, 2, 7), (2, 2, 9), (8, 2, 256), (8, 1, 8),
                                      (3, 4, 50), (8, 2, 0)])
def test_plan_indexing(nd, spd, n):
    dev, cx, slot = sva.multi_plan(nd, spd, n)
    j = np.arange(n)
    assert np.array_equal(dev, j % nd)
    assert np.array_equal(cx, (j // nd) % spd)
    # slots number each context's jobs 0, 1, 2, ... in job order
    for d in range(nd):
        for c in range(spd):
            mine = np.flatnonzero((dev == d) & (cx == c))
            assert np.array_equal(slot[mine], np.arange(len(mine)))
    # the load is balanced to within one pair per device and per context
    if n:
        per_dev = np.bincount(dev, minlength=nd)
        assert per_dev.max() - per_dev.min() <= 1
        per_ctx = np.bincount(dev * spd + cx, minlength=nd * spd)
        assert per_ctx.max() - per_ctx.min() <= 1


def test_plan_rejects_bad_shapes():
    for args in [(0, 1, 3), (1, 0, 3), (2, 2, -1)]:
        with pytest.raises(sva.SvaError):
            sva.multi_plan(*args)


def test_create_rejects_bad_device_lists():
    # invalid arguments are refused before the device count matters
    with pytest.raises(sva.SvaError) as e:
        sva.Multi([], 1)
    assert e.value.status == sva.SVA_ERR_INVALID_ARG
    with pytest.raises(sva.SvaError) as e:
        sva.Multi([0], 0)
    assert e.value.status == sva.SVA_ERR_INVALID_ARG


def test_config4_and_5_shard_shapes():
    """BASELINE config 4 at 8 GPUs: one TO_CENTER_SMALL pair per device; config
    5: 256 pairs -> 32 per device, 16 per stream with 2 streams."""
    dev, cx, _ = sva.multi_plan(8, 1, 8)
    assert sorted(dev.tolist()) == list(range(8))
    dev, cx, slot = sva.multi_plan(8, 2, 256)
    assert (np.bincount(dev) == 32).all()
    assert (np.bincount(dev * 2 + cx) == 16).all()
    assert slot.max() == 15
