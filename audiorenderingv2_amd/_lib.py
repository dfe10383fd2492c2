"""ctypes binding of libarx.so (include/arx.h).

The product path has no fallback: if the HIP library is missing or fails to load,
every entry point raises ArxError immediately.
"""
from __future__ import annotations

import ctypes as C
import os
import threading

_PKG = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(_PKG, "libarx.so")  # the product library (no environment override)

ARX_OK = 0
ABI_VERSION = 2  # include/arx.h ARX_ABI_VERSION
STATUS_NAMES = {
    0: "ARX_OK", 1: "ARX_ERR_INVALID_ARGUMENT", 2: "ARX_ERR_HIP", 3: "ARX_ERR_OUT_OF_MEMORY",
    4: "ARX_ERR_NOT_READY", 5: "ARX_ERR_IO", 6: "ARX_ERR_INTERNAL",
}


class ArxError(RuntimeError):
    def __init__(self, status: int, message: str):
        super().__init__(f"{STATUS_NAMES.get(status, status)}: {message}")
        self.status = status


class ArxConfig(C.Structure):
    _fields_ = [
        ("rays_x", C.c_int32), ("rays_y", C.c_int32), ("rays_z", C.c_int32),
        ("ir_length_in_seconds", C.c_uint32), ("sample_rate", C.c_int32),
        ("base_power", C.c_float), ("energy_thres", C.c_float), ("max_bounces", C.c_uint32),
        ("hrtf_absorption_rate", C.c_float), ("is_mono", C.c_int32), ("seed", C.c_uint64),
        ("device", C.c_int32),
    ]


class ArxStats(C.Structure):
    _fields_ = [
        ("queries", C.c_uint64), ("receiver_hits", C.c_uint64), ("misses", C.c_uint64),
        ("trace_ms", C.c_double), ("conv_ms", C.c_double),
        ("n_scene_tris", C.c_int64), ("n_receiver_tris", C.c_int64), ("n_nodes", C.c_int64),
        ("bvh_depth", C.c_int32),
        ("tree_hash", C.c_uint64), ("trace_vgprs", C.c_int32), ("trace_waves_per_simd", C.c_int32),
        ("trace_waves_target", C.c_int32), ("trace_format", C.c_int32),
        ("trace_grid_cus", C.c_int32),
    ]


PATH_MAX = 1024
NAME_MAX = 128
MAX_MATERIALS = 256


class ArxAppConfig(C.Structure):
    """arx_app_config: Context::loadContext's parameters (Context.cpp:15-164)."""
    _fields_ = [
        ("initial_volume", C.c_float),
        ("ir_length_in_seconds", C.c_uint32), ("width", C.c_uint32), ("height", C.c_uint32),
        ("write_first_ir_to_file", C.c_int32), ("write_first_output_to_file", C.c_int32),
        ("re_render_distance_threshold", C.c_float), ("re_render_angle_threshold", C.c_float),
        ("mono", C.c_int32),
        ("scene_file_path", C.c_char * PATH_MAX), ("audio_file_path", C.c_char * PATH_MAX),
        ("materials_file_path", C.c_char * PATH_MAX),
        ("initial_receiver_pos", C.c_float * 3), ("initial_emitter_pos", C.c_float * 3),
        ("base_power", C.c_float), ("rays", C.c_float * 3), ("ray_energy_threshold", C.c_float),
        ("ray_max_bounces", C.c_uint32), ("hrtf_absorption_rate", C.c_float),
        ("n_materials", C.c_int32),
        ("material_names", (C.c_char * NAME_MAX) * MAX_MATERIALS),
        ("material_absorption", C.c_float * MAX_MATERIALS),
    ]


_P = C.c_void_p
_F = C.POINTER(C.c_float)
_D = C.POINTER(C.c_double)
_I64 = C.POINTER(C.c_int64)
_I32 = C.POINTER(C.c_int32)

# arx_debug_share_scene's transport callbacks (include/arx.h)
SHARE_U64_FN = C.CFUNCTYPE(C.c_int, C.c_void_p, C.POINTER(C.c_uint64), C.c_int)
SHARE_BYTES_FN = C.CFUNCTYPE(C.c_int, C.c_void_p, C.POINTER(C.c_uint8), C.c_uint64)

# name -> (restype, argtypes); must cover every function declared in include/arx.h
SIGNATURES = {
    "arx_status_string": (C.c_char_p, [C.c_int]),
    "arx_last_error": (C.c_char_p, []),
    "arx_abi_version": (C.c_int, []),
    "arx_default_config": (None, [C.POINTER(ArxConfig)]),
    "arx_create": (C.c_int, [C.POINTER(ArxConfig), C.POINTER(_P)]),
    "arx_destroy": (None, [_P]),
    "arx_get_config": (C.c_int, [_P, C.POINTER(ArxConfig)]),
    "arx_set_stream": (C.c_int, [_P, _P]),
    "arx_get_stream": (_P, [_P]),
    "arx_set_scene": (C.c_int, [_P, _F, _F, C.c_int64]),
    "arx_set_receiver_model": (C.c_int, [_P, C.c_int, _F, C.c_int64]),
    "arx_place_receiver_vertices": (C.c_int, [_F, C.c_int64, C.c_float, C.c_float, C.c_float, C.c_float, _F]),
    "arx_material_absorption": (C.c_float, [C.c_char_p, C.POINTER(C.c_char_p), _F, C.c_size_t]),
    "arx_set_emitter": (C.c_int, [_P, C.c_float, C.c_float, C.c_float]),
    "arx_set_listener": (C.c_int, [_P, C.c_float, C.c_float, C.c_float, C.c_float]),
    "arx_set_thresholds": (C.c_int, [_P, C.c_float, C.c_uint32]),
    "arx_set_hrtf_absorption_rate": (C.c_int, [_P, C.c_float]),
    "arx_set_base_power": (C.c_int, [_P, C.c_float]),
    "arx_set_mono_output": (C.c_int, [_P, C.c_int]),
    "arx_set_seed": (C.c_int, [_P, C.c_uint64]),
    "arx_render": (C.c_int, [_P, _D]),
    "arx_set_frames_in_flight": (C.c_int, [_P, C.c_int32]),
    "arx_set_timing": (C.c_int, [_P, C.c_int32]),
    "arx_clear_histogram": (C.c_int, [_P]),
    "arx_trace_rays": (C.c_int, [_P, C.c_uint64, C.c_uint64]),
    "arx_histogram_device": (C.c_int, [_P, C.POINTER(_P), C.POINTER(C.c_size_t)]),
    "arx_finalize_ir": (C.c_int, [_P]),
    "arx_attach_histogram": (C.c_int, [_P, _P, C.c_size_t]),
    "arx_ir_device": (C.c_int, [_P, C.POINTER(_P), C.POINTER(_P), C.POINTER(C.c_size_t)]),
    "arx_copy_ir": (C.c_int, [_P, _F, _F, C.c_size_t]),
    "arx_get_stats": (C.c_int, [_P, C.POINTER(ArxStats)]),
    "arx_frac_bits": (C.c_int, [C.c_uint64]),
    "arx_set_ir": (C.c_int, [_P, _F, _F, C.c_size_t]),
    "arx_set_ir_device": (C.c_int, [_P, C.c_void_p, C.c_void_p, C.c_size_t]),
    "arx_convolute_audio_file": (C.c_int, [_P, _F, C.c_size_t, _F, _F, _D, _D]),
    "arx_convolute_device": (C.c_int, [_P, _P, C.c_size_t, _P, _P]),
    "arx_convolute_prepare_input": (C.c_int, [_P, _P, C.c_size_t]),
    "arx_convolute_prepared": (C.c_int, [_P, _P, _P, C.POINTER(C.c_size_t)]),
    "arx_convolute_live_block": (C.c_int, [_P, _D, C.c_size_t, _D, C.c_size_t]),
    "arx_convolute_live_device": (C.c_int, [_P, _P, C.c_size_t, _P]),
    "arx_prepare_ir_spectra": (C.c_int, [_P, C.c_int]),
    "arx_conv_describe": (C.c_int, [_P, C.c_int, C.c_char_p, C.c_size_t]),
    "arx_debug_ray_directions": (C.c_int, [C.c_uint64, C.c_uint64, C.c_uint64, _F, C.c_int]),
    "arx_debug_trace_counters": (C.c_int, [_P, C.POINTER(C.c_uint64), C.c_size_t]),
    "arx_debug_set_trace_path": (C.c_int, [_P, C.c_int]),
    "arx_debug_set_refit_pad": (C.c_int, [_P, C.c_float]),
    "arx_debug_check_tree_limits": (C.c_int, [C.c_uint64, C.c_uint64]),
    "arx_debug_wide_stats": (C.c_int, [_F, _F, C.c_int64, _F, C.c_int64, C.c_int32, C.c_uint64, _D, C.c_size_t]),
    "arx_debug_trace_profile": (C.c_int, [_P, C.POINTER(C.c_uint64), C.c_size_t, C.POINTER(C.c_size_t)]),
    "arx_debug_node_images": (C.c_int, [_P, _P, _P, C.c_size_t, _F, C.POINTER(C.c_uint64)]),
    "arx_trace_times": (C.c_int, [_P, _D, C.c_size_t, C.POINTER(C.c_size_t)]),
    "arx_conv_times": (C.c_int, [_P, _D, C.c_size_t, C.POINTER(C.c_size_t)]),
    "arx_live_times": (C.c_int, [_P, _D, C.c_size_t, C.POINTER(C.c_size_t)]),
    "arx_timing_ring": (C.c_int32, []),
    "arx_trace_kernel_id": (C.c_uint64, []),
    "arx_conv_kernel_id": (C.c_uint64, []),
    "arx_debug_set_leaf_max": (C.c_int, [C.c_int32]),
    "arx_device_count": (C.c_int32, []),
    "arx_device_alloc": (C.c_int, [C.c_int32, C.c_size_t, C.POINTER(_P)]),
    "arx_device_free": (None, [C.c_int32, _P]),
    "arx_memcpy": (C.c_int, [C.c_int32, _P, _P, C.c_size_t]),
    "arx_runtime_info": (C.c_int, [C.c_char_p, C.c_size_t]),
    "arx_scene_build_count": (C.c_uint64, []),
    "arx_debug_scene_roundtrip": (C.c_int, [_F, _F, C.c_int64, C.POINTER(C.c_uint64), C.POINTER(C.c_uint64)]),
    "arx_group_allreduce_f64": (C.c_int, [_P, _D, C.c_size_t, C.c_int]),
    "arx_stream_create": (C.c_int, [_P, C.c_int32, C.POINTER(_P)]),
    "arx_stream_destroy": (None, [_P]),
    "arx_stream_reset": (C.c_int, [_P]),
    "arx_stream_info": (C.c_int, [_P, _I32, _I32, _I32]),
    "arx_stream_process": (C.c_int, [_P, _D, C.c_size_t, _D, C.c_size_t]),
    "arx_stream_process_device": (C.c_int, [_P, C.c_void_p, C.c_size_t, C.c_void_p]),
    "arx_group_create": (C.c_int, [C.POINTER(ArxConfig), _I32, C.c_int32, C.POINTER(_P)]),
    "arx_group_unique_id": (C.c_int, [C.c_char_p, C.c_size_t]),
    "arx_group_create_rank": (C.c_int, [C.POINTER(ArxConfig), C.c_int32, C.c_int32, C.c_char_p, C.c_size_t,
                                        C.POINTER(_P)]),
    "arx_group_destroy": (None, [_P]),
    "arx_group_members": (C.c_int32, [_P]),
    "arx_group_ranks": (C.c_int32, [_P]),
    "arx_group_member": (_P, [_P, C.c_int32]),
    "arx_group_set_scene": (C.c_int, [_P, _F, _F, C.c_int64]),
    "arx_group_shard": (None, [C.c_uint64, C.c_int32, C.c_int32, C.POINTER(C.c_uint64), C.POINTER(C.c_uint64)]),
    "arx_debug_share_scene": (C.c_int, [C.c_int32, _F, _F, C.c_int64, SHARE_U64_FN, SHARE_BYTES_FN, _P,
                                        C.POINTER(C.c_uint64)]),
    "arx_group_set_receiver_model": (C.c_int, [_P, C.c_int, _F, C.c_int64]),
    "arx_group_set_emitter": (C.c_int, [_P, C.c_float, C.c_float, C.c_float]),
    "arx_group_set_listener": (C.c_int, [_P, C.c_float, C.c_float, C.c_float, C.c_float]),
    "arx_group_set_thresholds": (C.c_int, [_P, C.c_float, C.c_uint32]),
    "arx_group_set_hrtf_absorption_rate": (C.c_int, [_P, C.c_float]),
    "arx_group_set_base_power": (C.c_int, [_P, C.c_float]),
    "arx_group_set_mono_output": (C.c_int, [_P, C.c_int]),
    "arx_group_set_seed": (C.c_int, [_P, C.c_uint64]),
    "arx_group_render": (C.c_int, [_P, _D]),
    "arx_group_set_frames_in_flight": (C.c_int, [_P, C.c_int32]),
    "arx_group_set_timing": (C.c_int, [_P, C.c_int32]),
    "arx_group_allreduce_times": (C.c_int, [_P, C.c_int32, _D, C.c_size_t, C.POINTER(C.c_size_t)]),
    "arx_group_convolute_device": (C.c_int, [_P, C.POINTER(_P), C.c_size_t, C.POINTER(_P), C.POINTER(_P)]),
    "arx_group_conv_shard": (None, [C.c_int32, C.c_uint64, C.c_int32, C.c_int32, C.POINTER(C.c_uint64),
                                    C.POINTER(C.c_uint64)]),
    "arx_group_conv_sharded": (C.c_int32, [_P]),
    "arx_group_convolute_audio_file": (C.c_int, [_P, _F, C.c_size_t, _F, _F, _D, _D]),
    "arx_group_synchronize": (C.c_int, [_P]),
    "arx_group_copy_ir": (C.c_int, [_P, _F, _F, C.c_size_t]),
    "arx_group_get_stats": (C.c_int, [_P, C.POINTER(ArxStats)]),
    "arx_debug_group_force_collectives": (C.c_int, [_P, C.c_int32, C.c_int32]),
    "arx_debug_group_collectives": (C.c_int, [_P, C.POINTER(C.c_uint64)]),
    # input formats (host only)
    "arx_model_load_obj": (C.c_int, [C.c_char_p, C.c_char_p, C.c_int, C.c_char_p, C.POINTER(_P)]),
    "arx_model_free": (None, [_P]),
    "arx_model_mesh_count": (C.c_int64, [_P]),
    "arx_model_material_count": (C.c_int64, [_P]),
    "arx_model_info": (None, [_P, _I64, _I64, _I64]),
    "arx_model_mesh": (C.c_int, [_P, C.c_int64, C.POINTER(C.c_char_p), C.POINTER(_F), _I64,
                                 C.POINTER(_I32), _I64]),
    "arx_model_triangle_count": (C.c_int64, [_P]),
    "arx_model_flatten": (C.c_int, [_P, C.POINTER(C.c_char_p), _F, C.c_size_t, _F, _F]),
    "arx_wav_load": (C.c_int, [C.c_char_p, C.POINTER(_F), _I32, _I64, _I32, _I32]),
    "arx_free": (None, [_P]),
    "arx_wav_save": (C.c_int, [C.c_char_p, _F, C.c_int32, C.c_int64, C.c_int32, C.c_int32]),
    "arx_normalize_min_max": (C.c_int, [_F, C.c_size_t]),
    "arx_write_float_lines": (C.c_int, [C.c_char_p, _F, C.c_size_t]),
    "arx_default_app_config": (None, [C.POINTER(ArxAppConfig)]),
    "arx_parse_app_config": (C.c_int, [C.c_char_p, C.c_size_t, C.POINTER(ArxAppConfig)]),
    "arx_load_app_config": (C.c_int, [C.c_char_p, C.POINTER(ArxAppConfig)]),
}

_lib = None
_lock = threading.Lock()


def use_library(path: str) -> None:
    """Design tools only (tools/*.py): bind a design-experiment build (build.py --exp) instead of
    the product library; must precede the first call into the library."""
    global LIB_PATH
    with _lock:
        if _lib is not None:
            raise ArxError(6, "the library is already loaded")
        LIB_PATH = path


def lib() -> C.CDLL:
    """Load libarx.so once; raise (never fall back) if it is missing."""
    global _lib
    with _lock:
        if _lib is None:
            if not os.path.exists(LIB_PATH):
                raise ArxError(5, f"{LIB_PATH} not built: run `python -m audiorenderingv2_amd.build` "
                                  "(there is no CPU fallback for the HIP path)")
            handle = C.CDLL(LIB_PATH, mode=C.RTLD_GLOBAL)
            for name, (res, args) in SIGNATURES.items():
                fn = getattr(handle, name)
                fn.restype = res
                fn.argtypes = args
            if handle.arx_abi_version() != ABI_VERSION:
                raise ArxError(6, "ABI version mismatch")
            _lib = handle
        return _lib


def check(status: int) -> None:
    if status != ARX_OK:
        msg = lib().arx_last_error().decode(errors="replace")
        raise ArxError(status, msg)


def fptr(a) -> "C._Pointer":
    """float32 numpy array -> POINTER(c_float) (no copy)."""
    return a.ctypes.data_as(_F)
