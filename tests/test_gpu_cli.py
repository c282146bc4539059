"""The C++ CLI (rustraytrace_amd/rrt, mirroring main.rs:17-98) on the_next_week scenes that sample
the earth texture — 3 (earth), 9 (final_scene(800, 10000, 40)) and the default arm
(`_ => final_scene(400, 250, 4)`, the_next_week/mod.rs:68-81; no scene argument, 0 or any other
value) — with the texture resolved like RtwImage::new (rtw_image.rs:11-36): $RTW_IMAGES, the
working directory, images/ up to six parents, then the assets next to the executable. PPM bytes
must equal the Python API's render of the same scene.
"""
import os
import subprocess

import numpy as np
import pytest

import rustraytrace_amd as rrt

pytestmark = pytest.mark.gpu

CLI = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "rustraytrace_amd", "rrt")
KW = dict(image_width=48, samples_per_pixel=3, max_depth=6)


def _cli(args, path, env=None, cwd=None):
    r = subprocess.run([CLI, "--backend", "hip", "the_next_week", *args, "--image_width", "48", "--samples_per_pixel",
                        "3", "--max_depth", "6", "-o", str(path)], capture_output=True, text=True, env=env, cwd=cwd,
                       timeout=120)
    assert r.returncode == 0, r.stderr
    return r


def _python_ppm(scene_id, textures=None):
    sc = rrt.next_week_scene(scene_id, KW)
    assert len(sc.textures) == 1  # the scene samples the earth image
    if textures is not None:
        sc.textures = textures
    acc = rrt.render(sc)
    return rrt.format_ppm_from_accum(sc.width, sc.height, acc, sc.spp)


@pytest.mark.parametrize("args,scene_id", [(["3"], 3), (["9"], 9), ([], 10), (["0"], 10), (["17"], 10),
                                           (["+3"], 3), ([" 3"], 10), (["4294967297"], 10)])
def test_cli_earth_scenes_match_python(tmp_path, args, scene_id):
    path = tmp_path / "nw.ppm"
    r = _cli(args, path, cwd=str(tmp_path))
    assert "Could not load image file" not in r.stderr
    assert path.read_bytes() == _python_ppm(scene_id)


def test_cli_resolves_rtw_images_first(tmp_path):
    """$RTW_IMAGES/earthmap.ppm wins over the shipped asset (rtw_image.rs:14-19)."""
    rgb = np.zeros((4, 8, 3), np.uint8)
    rgb[:, :4] = (200, 30, 10)
    rgb[:, 4:] = (10, 40, 220)
    (tmp_path / "earthmap.ppm").write_bytes(b"P6\n8 4\n255\n" + rgb.tobytes())
    path = tmp_path / "nw.ppm"
    _cli(["3"], path, env=dict(os.environ, RTW_IMAGES=str(tmp_path)))
    assert path.read_bytes() == _python_ppm(3, textures=[rgb])
    assert path.read_bytes() != _python_ppm(3)
