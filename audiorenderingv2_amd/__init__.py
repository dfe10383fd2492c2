"""MI355X-native acoustic impulse-response engine (drop-in for AudioRenderingV2's GPU path).

libarx.so (HIP kernels + C ABI, include/arx.h) does the work; this package is the thin
Python host mirror of the reference's AudioRenderer plus scene/IO helpers.
"""
from ._lib import ArxError, LIB_PATH  # noqa: F401
from .renderer import AudioRenderer, DeviceBuffer, LiveStream, RenderGroup, RenderSettings, debug_ray_directions, device_count, frac_bits, place_receiver_vertices, runtime_info, scene_build_count  # noqa: F401
from .scene import Mesh, Scene, conference_standin, receiver_local, scene_from_meshes, test_obj_scene  # noqa: F401

__all__ = [
    "ArxError", "AudioRenderer", "DeviceBuffer", "LiveStream", "device_count", "runtime_info", "scene_build_count", "RenderGroup", "RenderSettings", "Scene", "Mesh", "conference_standin", "receiver_local",
    "scene_from_meshes", "test_obj_scene", "place_receiver_vertices", "debug_ray_directions", "frac_bits",
]
