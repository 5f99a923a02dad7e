"""The runtime's tunables (include/blsgpu.h blsgpu_set_option / blsgpu_get_option): every key documented there takes
a valid value and reads it back, out-of-range values and unknown keys are refused with ERR_ARGS and leave the value
unchanged, and the read-only properties cannot be written.  (The options' effect on results is covered by the parity
tests that force each form.)"""
import pytest

pytestmark = pytest.mark.gpu

# key -> (a valid non-default value, an invalid value or None)
KEYS = {
    "group_sets": (512, -1), "group_policy": (1, 2), "dedupe": (0, None), "merge_sets": (65536, -1),
    "miller_k": (2, 65), "miller_lanes": (3, 4), "miller_pairs": (1, 2), "lines_lanes": (1, 3),
    "msm_slice_mid": (64, 3), "msm_tree": (0, None), "f_run_max": (8, 3), "pipeline_depth": (2, 0),
    "merge_wait_us": (1000, -1), "idle_wait_us": (100, -1), "lane_tail_min": (1, -1), "lane_tail_parts": (1, 4),
    "merge_balance": (1, None), "early_release": (1, None), "tail_on_msg": (1, None), "copy_stream": (1, None),
    "coop_max": (256, -1), "coop_g2_max": (1024, -1), "coop_excl_max": (128, -1), "rsig_spec": (0, None), "spec_large": (0, None), "spec_gsm": (1, None),
    "fb_lane_min": (64, -1), "fb_direct_min": (512, -1), "fb_check6": (1, 3), "fb_force_busy": (1, None), "keep_f": (0, None), "keep_copy": (1, None),
    "route_split_sets": (8192, 0), "acc6_max": (4096, -1), "small_max": (2048, -1), "serial": (1, None),
    "profile": (1, None), "max_devices": (1, 0),
    "urgent_lane": (0, None), "urgent_max_sets": (64, -1), "urgent_excl": (1, None), "urgent_wait_us": (0, -1), "group_adapt": (0, None),
    # stream creation options: the fixture's context has made no call yet, so they still take values
    "urgent_cus": (16, 12), "urgent_isolate": (2, 4), "blocking_sync": (0, 2), "pipeline_prio": (0, 2),
}


@pytest.fixture(scope="module")
def ctx():
    from lodestar_amd.native import Context

    c = Context([0])
    yield c
    c.close()


@pytest.mark.parametrize("key", sorted(KEYS))
def test_option_roundtrip(ctx, key):
    good, bad = KEYS[key]
    old = ctx.get_option(key)
    try:
        ctx.set_option(key, good)
        assert ctx.get_option(key) == good
        if bad is not None:
            with pytest.raises(ValueError):
                ctx.set_option(key, bad)
            assert ctx.get_option(key) == good
    finally:
        ctx.set_option(key, old)
    assert ctx.get_option(key) == old


def test_unknown_and_read_only_keys(ctx):
    with pytest.raises(ValueError):
        ctx.set_option("no_such_option", 1)
    with pytest.raises(ValueError):
        ctx.get_option("no_such_option")
    for ro in ("hw_queues", "abi_version"):
        v = ctx.get_option(ro)
        assert v > 0
        with pytest.raises(ValueError):
            ctx.set_option(ro, v + 1)
    assert ctx.get_option("spurious_groups") == 0
    with pytest.raises(ValueError):
        ctx.set_option("spurious_groups", 1)
