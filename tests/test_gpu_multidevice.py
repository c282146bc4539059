"""The drop-in's in-library multi-device path (rrt_hip_render with n_gpus > 1: one host thread per
device, row bands dealt in serpentine order, each device's bands copied straight into the caller's image by
a strided 2-D copy plus one plain copy of a partial last band; rrt_host.cpp render_frame) run with
more than one worker on a one-GPU box: the test-only entry point rrt_testing_device_wrap(1) maps
worker g to device g % device_count, so 2, 3 and 8 workers share the GPU and every copy path runs.
The frame is 100x56 (bands of 16: 16, 16, 16, 8 rows), so the partial last band, workers with two
bands and workers with none (8 workers) all occur; a 240x135 frame (9 bands) gives every worker of
2 and 3 several bands per serpentine parity, so the strided copies' 2 x n_ranks-band pitch moves
more than one band. Every image must be bit-identical to n_gpus = 1: a pixel's samples are keyed
by its global index (include/rrt_hip.h), whatever worker renders it.
"""
import numpy as np
import pytest

import rustraytrace_amd as rrt

pytestmark = pytest.mark.gpu


@pytest.fixture
def wrap():
    lib = rrt._lib.load()
    lib.rrt_testing_device_wrap(1)
    yield
    lib.rrt_testing_device_wrap(0)


def _scene():
    sc = rrt.rtow(image_width=100, samples_per_pixel=6, max_depth=10)
    assert sc.height == 56
    return sc


@pytest.mark.parametrize("n", [2, 3, 8])
def test_float_accum_bit_identical_to_one_device(wrap, n):
    sc = _scene()
    one = rrt.render(sc, n_gpus=1)
    many = rrt.render(sc, n_gpus=n)
    assert np.array_equal(one, many)
    assert np.all(many[..., 3] == sc.spp)


@pytest.mark.parametrize("n", [2, 3])
def test_tall_frame_several_bands_per_parity(wrap, n):
    sc = rrt.rtow(image_width=240, samples_per_pixel=4, max_depth=10)
    assert sc.height == 135  # 9 bands of 16 (the last 7 rows): 2 workers own 5 / 4 bands, 3 own 3 each
    one = rrt.render(sc, n_gpus=1)
    assert np.array_equal(one, rrt.render(sc, n_gpus=n))
    assert np.array_equal(rrt.render_rgb8(sc, n_gpus=1), rrt.render_rgb8(sc, n_gpus=n))
    assert np.array_equal(rrt.render_f64(sc, n_gpus=1), rrt.render_f64(sc, n_gpus=n))


@pytest.mark.parametrize("n", [2, 3, 8])
def test_rgb8_bit_identical_to_one_device(wrap, n):
    sc = _scene()
    assert np.array_equal(rrt.render_rgb8(sc, n_gpus=1), rrt.render_rgb8(sc, n_gpus=n))


@pytest.mark.parametrize("n", [3, 8])
def test_f64_bit_identical_to_one_device(wrap, n):
    sc = _scene()
    assert np.array_equal(rrt.render_f64(sc, n_gpus=1), rrt.render_f64(sc, n_gpus=n))


def test_progress_lines_with_several_workers(wrap, capfd):
    sc = _scene()
    one = rrt.render(sc, n_gpus=1)
    many = rrt.render(sc, n_gpus=3, quiet=False)
    err = capfd.readouterr().err
    assert "(3/3 GPUs done)" in err and "100%" in err
    assert np.array_equal(one, many)


def test_more_workers_than_devices_is_refused_without_the_test_mode():
    sc = _scene()
    n = rrt.device_count() + 1
    with pytest.raises(rrt.RrtError, match="visible devices"):
        rrt.render(sc, n_gpus=n)
