"""rustraytrace_amd — MI355X (gfx950) HIP path-tracing backend for jwheo12/RustRayTrace.

The product is librrt_hip.so (rustraytrace_amd/csrc: gfx950 megakernel + host runtime +
C-ABI declared in include/rrt_hip.h). This package is the Python host over that C-ABI:
scene builders, render entries, PPM output. It never renders on the CPU.
"""
from . import _lib, world
from ._lib import RrtError, load
from .render import (
    DeviceScene,
    device_count,
    format_pnm_from_rgb8,
    format_ppm_from_accum,
    quantize_accum,
    quantize_accum_books,
    quantize_accum_books_f64,
    quantize_accum_async,
    render,
    render_f64,
    render_in_one_weekend,
    render_rgb8,
    write_pnm_from_rgb8,
    write_ppm_from_accum,
)
from .scenes import (
    CONFIGS,
    SceneData,
    build_in_one_weekend_scene,
    config_scene,
    named_scene,
    earth_light,
    earth_texture,
    next_week_scene,
    rest_of_your_life_scene,
    make_camera,
    rtow,
    three_spheres,
)

__all__ = [
    "_lib", "RrtError", "load", "DeviceScene", "device_count", "format_ppm_from_accum", "quantize_accum", "quantize_accum_books", "quantize_accum_books_f64", "render", "render_f64",
    "render_in_one_weekend", "write_ppm_from_accum", "render_rgb8", "quantize_accum_async", "format_pnm_from_rgb8",
    "write_pnm_from_rgb8", "CONFIGS", "SceneData", "build_in_one_weekend_scene",
    "config_scene", "named_scene", "earth_light", "earth_texture", "next_week_scene", "rest_of_your_life_scene", "make_camera", "rtow", "three_spheres",
]
