"""ctypes binding of libphdslam.so (the C-ABI in include/phd_capi.h).

The library is loaded from this package directory (built in-tree by
cuda-phdslam_amd/build.py).  There is no fallback: if the .so is missing the
import of any compute entry point raises, loudly.
"""
import ctypes
import os

from .types import AckermanControl, Capacity, SlamConfig

_HERE = os.path.dirname(os.path.abspath(__file__))
# PHDSLAM_LIB selects an alternative in-tree build (e.g. the PHD_STAMPS diagnostic build)
LIB_PATH = os.environ.get("PHDSLAM_LIB") or os.path.join(_HERE, "libphdslam.so")

PHD_OK = 0
PHD_E_ARG = -1
PHD_E_HIP = -2
PHD_E_CAPACITY = -3
PHD_E_UNSUPPORTED = -4
PHD_E_NODEVICE = -5

_c_int_p = ctypes.POINTER(ctypes.c_int)
_c_float_p = ctypes.POINTER(ctypes.c_float)
_vp = ctypes.c_void_p
_u64 = ctypes.c_uint64

# name -> (restype, argtypes)
SIGNATURES = {
    "phd_version": (ctypes.c_char_p, []),
    "phd_last_error": (ctypes.c_char_p, []),
    "phd_device_count": (ctypes.c_int, [_c_int_p]),
    "phd_ctx_create": (ctypes.c_int, [ctypes.POINTER(_vp), ctypes.c_int, ctypes.c_int, ctypes.POINTER(Capacity)]),
    "phd_ctx_destroy": (ctypes.c_int, [_vp]),
    "phd_ctx_info": (ctypes.c_int, [_vp, _c_int_p, ctypes.POINTER(Capacity)]),
    "phd_set_config": (ctypes.c_int, [_vp, ctypes.POINTER(SlamConfig)]),
    "phd_set_stream": (ctypes.c_int, [_vp, _vp]),
    "phd_get_stream": (_vp, [_vp]),
    "phd_synchronize": (ctypes.c_int, [_vp]),
    "phd_set_seed": (ctypes.c_int, [_vp, _u64]),
    "phd_load_particles": (ctypes.c_int, [_vp, ctypes.c_int, _vp, _vp, _vp, _vp]),
    "phd_export_particles": (ctypes.c_int, [_vp, ctypes.c_int, _vp, _vp, _vp]),
    "phd_export_maps": (ctypes.c_int, [_vp, ctypes.c_int, _vp, _vp]),
    "phd_slab_sizes": (ctypes.c_int, [_vp, _vp]),
    "phd_enable_dynamic": (ctypes.c_int, [_vp, ctypes.c_int]),
    "phd_load_dynamic_maps": (ctypes.c_int, [_vp, ctypes.c_int, _vp, _vp]),
    "phd_dynamic_sizes": (ctypes.c_int, [_vp, _vp]),
    "phd_export_dynamic_maps": (ctypes.c_int, [_vp, ctypes.c_int, _vp, _vp]),
    "phd_predict_dynamic": (ctypes.c_int, [_vp]),
    "phd_set_poses": (ctypes.c_int, [_vp, ctypes.c_int, _vp]),
    "phd_predict_ackerman": (ctypes.c_int, [_vp, AckermanControl, _vp, _u64]),  # struct by value
    "phd_predict_cv": (ctypes.c_int, [_vp, _vp, _u64]),
    "phd_set_measurements": (ctypes.c_int, [_vp, _vp, ctypes.c_int]),
    "phd_update": (ctypes.c_int, [_vp]),
    "phd_normalize": (ctypes.c_int, [_vp, _c_float_p]),
    "phd_neff": (ctypes.c_int, [_vp, _c_float_p]),
    "phd_resample": (ctypes.c_int, [_vp, _vp, _u64, _vp]),
    "phd_step": (ctypes.c_int, [_vp, _vp, ctypes.c_int, _u64, _c_float_p, _c_int_p]),
    "phd_resample_count": (ctypes.c_int, [_vp, _c_int_p]),
    "phd_cardinality_distribution": (ctypes.c_int, [_vp, _vp]),
    "phd_predict_update": (ctypes.c_int, [_vp, _vp, ctypes.c_int, _u64, _vp]),
    "phd_copy_log_weights": (ctypes.c_int, [_vp, _vp]),
    "phd_set_log_weights": (ctypes.c_int, [_vp, _vp]),
    "phd_apply_resample": (ctypes.c_int, [_vp, _vp, ctypes.c_float]),
    "phd_global_resample": (ctypes.c_int, [_vp, _vp, ctypes.c_int, ctypes.c_int, _u64, _u64, _vp, _c_float_p,
                                           _c_int_p]),
    "phd_shard_resample": (ctypes.c_int, [_vp, _vp, ctypes.c_int, ctypes.c_int, _u64, _u64, _vp, _vp, _vp, _vp, _vp,
                                          ctypes.c_int, ctypes.c_float, _c_int_p, _c_int_p, _c_int_p, _c_float_p,
                                          _c_int_p]),
    "phd_shard_receive": (ctypes.c_int, [_vp, _vp, _vp, ctypes.c_int, ctypes.c_int]),
    "phd_shard_resample_async": (ctypes.c_int, [_vp, _vp, ctypes.c_int, ctypes.c_int, _u64, _u64, _vp, _vp, _vp, _vp,
                                                _vp, ctypes.c_int, _vp, ctypes.c_int, ctypes.c_float]),
    "phd_shard_receive_blocks": (ctypes.c_int, [_vp, _vp, ctypes.c_int, _vp]),
    "phd_shard_poll": (ctypes.c_int, [_vp, _vp, _vp, _vp, _vp, _vp, _vp]),
    "phd_shard_receive_overflow": (ctypes.c_int, [_vp, _vp, ctypes.c_int, _vp]),
    "phd_update_pending": (ctypes.c_int, [_vp, _vp, ctypes.c_int, _u64, _vp]),
    "phd_add_births": (ctypes.c_int, [_vp, _vp, ctypes.c_int]),
    "phd_set_step_births": (ctypes.c_int, [_vp, ctypes.c_int]),
    "phd_wait_logw": (ctypes.c_int, [_vp, _vp]),
    "phd_set_edge_pool": (ctypes.c_int, [_vp, ctypes.c_int]),
    "phd_set_pair_list_cap": (ctypes.c_int, [_vp, ctypes.c_int]),
    "phd_set_plan_stream": (ctypes.c_int, [_vp, _vp]),
    "phd_step_births": (ctypes.c_int, [_vp, _vp]),
    "phd_set_index_offset": (ctypes.c_int, [_vp, ctypes.c_int]),
    "phd_fill_log_weights": (ctypes.c_int, [_vp, ctypes.c_float]),
    "phd_record_bytes": (ctypes.c_int, [_vp, ctypes.POINTER(ctypes.c_size_t)]),
    "phd_pack_particles": (ctypes.c_int, [_vp, _vp, ctypes.c_int, _vp]),
    "phd_unpack_particles": (ctypes.c_int, [_vp, _vp, _vp, ctypes.c_int]),
    "phd_expected_pose": (ctypes.c_int, [_vp, _vp, _c_int_p]),
    "phd_cardinalities": (ctypes.c_int, [_vp, _vp]),
    "phd_expected_map": (ctypes.c_int, [_vp, _vp, ctypes.c_long, ctypes.POINTER(ctypes.c_long)]),
    "phd_expected_map_dynamic": (ctypes.c_int, [_vp, _vp, ctypes.c_long, ctypes.POINTER(ctypes.c_long)]),
    # host-only I/O (include/phd_io.h)
    "phd_load_timestamps": (ctypes.c_int, [ctypes.c_char_p, _vp, ctypes.c_int, _c_int_p]),
    "phd_load_controls": (ctypes.c_int, [ctypes.c_char_p, ctypes.c_int, _vp, ctypes.c_int, _c_int_p]),
    "phd_load_measurements": (ctypes.c_int, [ctypes.c_char_p, ctypes.c_int, _vp, ctypes.c_long, _vp, ctypes.c_int,
                                             _c_int_p]),
    "phd_write_state_log": (ctypes.c_int, [ctypes.c_char_p, ctypes.c_int, _vp, _vp, ctypes.c_long, _vp, _vp,
                                           ctypes.c_int, _vp, _vp, ctypes.c_int, ctypes.c_int, ctypes.c_int]),
    "phd_expected_map_groups": (ctypes.c_int, [_vp, _c_int_p]),
    "phd_last_update_ms": (ctypes.c_int, [_vp, _c_float_p]),
    "phd_enable_timing": (ctypes.c_int, [_vp, ctypes.c_int]),
    "phd_set_timing_stride": (ctypes.c_int, [_vp, ctypes.c_int]),
    "phd_update_timing": (ctypes.c_int, [_vp, _c_float_p, _c_int_p]),
    "phd_set_replay": (ctypes.c_int, [_vp, ctypes.c_int]),
    "phd_lse_parts": (ctypes.c_int, [_vp, _vp]),
    "phd_set_check_each_update": (ctypes.c_int, [_vp, ctypes.c_int]),
    "phd_check_errors": (ctypes.c_int, [_vp]),
    "phd_set_merge_mode": (ctypes.c_int, [_vp, ctypes.c_int]),
    "phd_set_update_threads": (ctypes.c_int, [_vp, ctypes.c_int]),
    "phd_update_threads": (ctypes.c_int, [_vp, _c_int_p, ctypes.POINTER(ctypes.c_size_t), _c_int_p]),
    "phd_set_update_form": (ctypes.c_int, [_vp, ctypes.c_int]),
    "phd_update_form": (ctypes.c_int, [_vp, _c_int_p]),
    "phd_debug_stamps": (ctypes.c_int, [_vp, _vp, ctypes.c_int]),
    "phd_merge_fallbacks": (ctypes.c_int, [_vp, _c_int_p]),
    "phd_merge_pair_overflows": (ctypes.c_int, [_vp, _c_int_p]),
    "phd_status_errors": (ctypes.c_int, [_vp, _c_int_p]),
    "phd_particle_status": (ctypes.c_int, [_vp, _vp]),
    "phd_config_defaults": (ctypes.c_int, [ctypes.POINTER(SlamConfig)]),
    "phd_config_load": (ctypes.c_int, [ctypes.c_char_p, ctypes.POINTER(SlamConfig), ctypes.c_char_p, ctypes.c_int]),
    "phd_synth_preset": (ctypes.c_int, [ctypes.c_int, ctypes.POINTER(SlamConfig), _c_int_p, _c_int_p, _c_int_p,
                                        _c_float_p]),
    "phd_synth_scenario": (ctypes.c_int, [ctypes.POINTER(SlamConfig), ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                          ctypes.c_float, _u64, _vp, _vp, _vp, _vp, _vp]),
}

_lib = None


class PHDError(RuntimeError):
    def __init__(self, code, where, msg):
        super().__init__(f"{where} failed with code {code}: {msg}")
        self.code = code


def lib():
    """Load libphdslam.so (raises if it has not been built)."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise OSError(f"{LIB_PATH} not found: build it with `python cuda-phdslam_amd/build.py` "
                          "(the HIP path has no CPU fallback)")
        # One HIP runtime per process: torch bundles its own libamdhip64.so.7.
        # Loaded first, it also serves libphdslam.so's NEEDED entry (same
        # soname); loaded second, a second runtime would find no devices.
        try:
            import torch  # noqa: F401
        except ImportError:
            pass
        L = ctypes.CDLL(LIB_PATH)
        for name, (res, args) in SIGNATURES.items():
            fn = getattr(L, name)
            fn.restype = res
            fn.argtypes = args
        _lib = L
    return _lib


def check(rc, where):
    if rc != PHD_OK:
        msg = lib().phd_last_error()
        raise PHDError(rc, where, msg.decode() if msg else "")
    return rc


def device_count():
    c = ctypes.c_int(0)
    check(lib().phd_device_count(ctypes.byref(c)), "phd_device_count")
    return c.value
