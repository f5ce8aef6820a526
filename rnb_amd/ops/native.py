"""ctypes bindings for the in-tree native libraries (rnb_amd/_native/*.so).

Design note: the HIP libraries export a plain C ABI and are loaded with
ctypes instead of being compiled as PyTorch C++ extensions. They build with a
single ``hipcc`` call in seconds, carry no PyTorch-ABI coupling, and launch on
whatever ``hipStream_t`` the caller passes (``torch.cuda.current_stream()
.cuda_stream``), which is what HIP-graph capture needs.

Loading policy: on a machine with a visible GPU a missing or stale library is
a hard error (``NativeUnavailable``) -- the GPU path never silently falls
back to PyTorch. On a CPU-only machine callers may probe ``available()``.
"""
from __future__ import annotations

import ctypes
import os
import threading
from typing import Optional

_HERE = os.path.dirname(os.path.abspath(__file__))
NATIVE_DIR = os.path.join(os.path.dirname(_HERE), "_native")

_lock = threading.Lock()
_libs = {}


class NativeUnavailable(RuntimeError):
    pass


def _lib_path(name: str) -> str:
    return os.path.join(NATIVE_DIR, name)


def _load(name: str, build_if_missing: bool = True) -> ctypes.CDLL:
    with _lock:
        lib = _libs.get(name)
        if lib is not None:
            return lib
        path = _lib_path(name)
        if not os.path.exists(path) and build_if_missing and \
                os.environ.get("RNB_NO_AUTOBUILD") != "1":
            from .. import build
            try:
                build.build_one(name)
            except Exception as err:  # pragma: no cover - reported below
                raise NativeUnavailable("could not build %s: %s" % (name, err))
        if not os.path.exists(path):
            raise NativeUnavailable("%s not built; run `python -m rnb_amd.build`"
                                    % path)
        try:
            lib = ctypes.CDLL(path, mode=ctypes.RTLD_GLOBAL)
        except OSError as err:
            raise NativeUnavailable("failed to load %s: %s" % (path, err))
        _libs[name] = lib
        return lib


def available(name: str = "librnb_kernels.so") -> bool:
    try:
        _load(name)
        return True
    except NativeUnavailable:
        return False


def loaded_paths():
    """Paths of the native libraries loaded into this process."""
    return sorted(_lib_path(n) for n in _libs)


def _check(rc: int, what: str, lib: Optional[ctypes.CDLL] = None) -> None:
    if rc == 0:
        return
    if rc < 0:
        raise RuntimeError("%s: shape/contract check failed (code %d)" % (what, rc))
    msg = ""
    try:
        rt = _load("librnb_runtime.so")
        rt.rnb_error_string.restype = ctypes.c_char_p
        msg = rt.rnb_error_string(rc).decode()
    except Exception:
        pass
    raise RuntimeError("%s failed: hipError %d %s" % (what, rc, msg))


# ---------------------------------------------------------------------------
# kernels
# ---------------------------------------------------------------------------
class ConvParams(ctypes.Structure):
    """Mirror of ``struct ConvParams`` in csrc/conv_igemm.hip."""
    _fields_ = [
        ("x", ctypes.c_void_p), ("w", ctypes.c_void_p), ("bias", ctypes.c_void_p),
        ("res", ctypes.c_void_p), ("y", ctypes.c_void_p),
        ("N", ctypes.c_int), ("T", ctypes.c_int), ("H", ctypes.c_int),
        ("W", ctypes.c_int), ("Cin_p", ctypes.c_int),
        ("To", ctypes.c_int), ("Ho", ctypes.c_int), ("Wo", ctypes.c_int),
        ("KT", ctypes.c_int), ("KH", ctypes.c_int), ("KW", ctypes.c_int),
        ("ST", ctypes.c_int), ("SH", ctypes.c_int), ("SW", ctypes.c_int),
        ("PT", ctypes.c_int), ("PH", ctypes.c_int), ("PW", ctypes.c_int),
        ("Cout_p", ctypes.c_int), ("y_stride", ctypes.c_int),
        ("res_stride", ctypes.c_int), ("K_total", ctypes.c_int),
        ("K_pad", ctypes.c_int), ("M", ctypes.c_int), ("relu", ctypes.c_int),
        ("n_ptiles", ctypes.c_int), ("n_ctiles", ctypes.c_int),
        ("x_bytes", ctypes.c_uint32), ("w_rows", ctypes.c_int),
        ("ktab", ctypes.c_void_p),
        ("mWo", ctypes.c_uint32), ("sWo", ctypes.c_uint32),
        ("mHo", ctypes.c_uint32), ("sHo", ctypes.c_uint32),
        ("mTo", ctypes.c_uint32), ("sTo", ctypes.c_uint32),
        ("row_mode", ctypes.c_int), ("ngroups", ctypes.c_int),
        ("mG", ctypes.c_uint32), ("sG", ctypes.c_uint32),
    ]


class HaloParams(ctypes.Structure):
    """Mirror of ``struct HaloParams`` in csrc/conv_halo.hip."""
    _fields_ = [
        ("x", ctypes.c_void_p), ("w", ctypes.c_void_p), ("bias", ctypes.c_void_p),
        ("res", ctypes.c_void_p), ("y", ctypes.c_void_p),
        ("frames", ctypes.c_int), ("H", ctypes.c_int), ("W", ctypes.c_int),
        ("Cin", ctypes.c_int), ("Cout_p", ctypes.c_int), ("y_stride", ctypes.c_int),
        ("res_stride", ctypes.c_int), ("K_pad", ctypes.c_int), ("M", ctypes.c_int),
        ("relu", ctypes.c_int), ("w_rows", ctypes.c_int), ("n_ptiles", ctypes.c_int),
        ("n_ctiles", ctypes.c_int), ("R", ctypes.c_int), ("bands", ctypes.c_int),
        ("np", ctypes.c_int), ("x_bytes", ctypes.c_uint32),
        ("mB", ctypes.c_uint32), ("sB", ctypes.c_uint32), ("mW", ctypes.c_uint32),
        ("sW", ctypes.c_uint32),
    ]


class Conv21Params(ctypes.Structure):
    """Mirror of ``struct Conv21Params`` in csrc/conv21.hip."""
    _fields_ = [
        ("x", ctypes.c_void_p), ("ws", ctypes.c_void_p), ("bs", ctypes.c_void_p),
        ("wt", ctypes.c_void_p), ("bt", ctypes.c_void_p), ("res", ctypes.c_void_p),
        ("y", ctypes.c_void_p),
        ("N", ctypes.c_int), ("T", ctypes.c_int), ("H", ctypes.c_int), ("W", ctypes.c_int),
        ("ks_pad", ctypes.c_int), ("y_stride", ctypes.c_int), ("res_stride", ctypes.c_int),
        ("relu", ctypes.c_int), ("n_units", ctypes.c_int), ("bands", ctypes.c_int),
        ("x_bytes", ctypes.c_uint32), ("mB", ctypes.c_uint32), ("sB", ctypes.c_uint32),
        ("mW", ctypes.c_uint32), ("sW", ctypes.c_uint32),
    ]


class WinoParams(ctypes.Structure):
    """Mirror of ``struct WinoParams`` in csrc/wino_common.h."""
    _fields_ = [
        ("x", ctypes.c_void_p), ("u", ctypes.c_void_p), ("bias", ctypes.c_void_p),
        ("res", ctypes.c_void_p), ("y", ctypes.c_void_p),
        ("F", ctypes.c_int), ("H", ctypes.c_int), ("W", ctypes.c_int), ("Cin", ctypes.c_int),
        ("Cout", ctypes.c_int), ("y_stride", ctypes.c_int), ("res_stride", ctypes.c_int),
        ("relu", ctypes.c_int), ("tiles_h", ctypes.c_int), ("tiles_w", ctypes.c_int),
        ("n_tiles", ctypes.c_int), ("n_tblocks", ctypes.c_int), ("n_cblocks", ctypes.c_int),
        ("x_bytes", ctypes.c_uint32), ("u_bytes", ctypes.c_uint32),
        ("m_tw", ctypes.c_uint32), ("s_tw", ctypes.c_uint32),
        ("m_th", ctypes.c_uint32), ("s_th", ctypes.c_uint32),
        ("in_ss", ctypes.c_void_p), ("clip_seg", ctypes.c_void_p),
        ("out_stats", ctypes.c_void_p), ("clip_frames", ctypes.c_int), ("stats_c", ctypes.c_int),
    ]


class TemporalParams(ctypes.Structure):
    """Mirror of ``struct TemporalParams`` in csrc/conv_temporal.hip."""
    _fields_ = [
        ("x", ctypes.c_void_p), ("w", ctypes.c_void_p), ("bias", ctypes.c_void_p),
        ("res", ctypes.c_void_p), ("y", ctypes.c_void_p),
        ("N", ctypes.c_int), ("T", ctypes.c_int), ("HW", ctypes.c_int),
        ("Cin_p", ctypes.c_int), ("Cout_p", ctypes.c_int), ("y_stride", ctypes.c_int),
        ("res_stride", ctypes.c_int), ("K_pad", ctypes.c_int), ("relu", ctypes.c_int),
        ("w_rows", ctypes.c_int), ("ngroups", ctypes.c_int), ("gpc", ctypes.c_int),
        ("n_ctiles", ctypes.c_int), ("x_bytes", ctypes.c_uint32),
        ("mG", ctypes.c_uint32), ("sG", ctypes.c_uint32),
    ]


class Kernels:
    """Typed wrappers over librnb_kernels.so."""

    def __init__(self):
        lib = _load("librnb_kernels.so")
        self.lib = lib
        lib.rnb_conv_num_configs.restype = ctypes.c_int
        lib.rnb_conv_config_info.argtypes = [ctypes.c_int, ctypes.POINTER(ctypes.c_int),
                                             ctypes.POINTER(ctypes.c_int)]
        lib.rnb_conv_params_size.restype = ctypes.c_int
        lib.rnb_conv_launch.argtypes = [ctypes.POINTER(ConvParams), ctypes.c_int,
                                        ctypes.c_void_p]
        lib.rnb_conv_launch.restype = ctypes.c_int
        lib.rnb_clipgen_u8.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                                       ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                       ctypes.c_int, ctypes.c_void_p]
        lib.rnb_clipgen_video.argtypes = [ctypes.c_void_p, ctypes.c_int,
                                          ctypes.POINTER(ctypes.c_int), ctypes.c_int,
                                          ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                          ctypes.c_void_p]
        lib.rnb_nv12gen_video.argtypes = [ctypes.c_void_p, ctypes.c_int,
                                          ctypes.POINTER(ctypes.c_int), ctypes.c_int,
                                          ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                          ctypes.c_void_p]
        lib.rnb_nv12gen.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                                    ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                    ctypes.c_void_p]
        lib.rnb_nv12_to_clip.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_longlong,
                                         ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                         ctypes.c_int, ctypes.POINTER(ctypes.c_float),
                                         ctypes.POINTER(ctypes.c_float),
                                         ctypes.POINTER(ctypes.c_float), ctypes.c_int,
                                         ctypes.c_void_p]
        lib.rnb_preprocess.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_longlong,
                                       ctypes.POINTER(ctypes.c_float),
                                       ctypes.POINTER(ctypes.c_float), ctypes.c_void_p]
        lib.rnb_stem_pack.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_longlong,
                                      ctypes.c_int, ctypes.c_int, ctypes.c_void_p]
        lib.rnb_preprocess_packed.argtypes = [ctypes.c_void_p, ctypes.c_void_p,
                                              ctypes.c_longlong, ctypes.c_int, ctypes.c_int,
                                              ctypes.POINTER(ctypes.c_float),
                                              ctypes.POINTER(ctypes.c_float), ctypes.c_void_p]
        lib.rnb_head.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                                 ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int, ctypes.c_int,
                                 ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_void_p]
        lib.rnb_bn_scratch_floats.argtypes = [ctypes.c_int, ctypes.c_int]
        lib.rnb_bn_scratch_floats.restype = ctypes.c_longlong
        lib.rnb_bn_stats.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                     ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                                     ctypes.c_void_p]
        lib.rnb_bn_apply.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                                     ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                                     ctypes.c_void_p, ctypes.c_float, ctypes.c_int,
                                     ctypes.c_longlong, ctypes.c_int, ctypes.c_int,
                                     ctypes.c_int, ctypes.c_int, ctypes.c_void_p]
        lib.rnb_bn_seg_bps.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_longlong]
        lib.rnb_bn_seg_set_bps.argtypes = [ctypes.c_int]
        if os.environ.get("RNB_BN_BPS"):
            # fixed BN statistics blocks per segment (batch-invariant split)
            lib.rnb_bn_seg_set_bps(int(os.environ["RNB_BN_BPS"]))
        lib.rnb_bn_aff_arm.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p,
                                       ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_void_p,
                                       ctypes.c_void_p, ctypes.c_float, ctypes.c_void_p]
        lib.rnb_bn_aff_arm.restype = ctypes.c_int
        lib.rnb_bn_aff_disarm.argtypes = []
        lib.rnb_bn_aff_disarm.restype = None
        lib.rnb_bn_aff_used.argtypes = []
        lib.rnb_bn_aff_used.restype = ctypes.c_int
        lib.rnb_bn_set_apply_blk.argtypes = [ctypes.c_int]
        lib.rnb_bn_set_apply_blk.restype = None
        if "RNB_BN_APPLY_BLK" in os.environ:
            # block-tiled BN applies (default 1; 0: the per-thread-row kernels)
            lib.rnb_bn_set_apply_blk(int(os.environ["RNB_BN_APPLY_BLK"]))
        lib.rnb_bn_seg_set_fused_finalize.argtypes = [ctypes.c_int]
        if os.environ.get("RNB_BN_FUSED_FINALIZE"):
            # fused finalize + running-update kernel up to this many videos
            # per launch (default 32; 0: separate kernels, A/B)
            lib.rnb_bn_seg_set_fused_finalize(int(os.environ["RNB_BN_FUSED_FINALIZE"]))
        lib.rnb_bn_seg_scratch_floats.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_longlong]
        lib.rnb_bn_seg_scratch_floats.restype = ctypes.c_longlong
        lib.rnb_bn_seg_stats_f32.argtypes = [
            ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_longlong,
            ctypes.c_int, ctypes.c_int, ctypes.c_void_p, ctypes.c_longlong,
            ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_float, ctypes.c_float,
            ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
            ctypes.c_void_p, ctypes.c_void_p]
        lib.rnb_bn_seg_stats_from_sums_f32.argtypes = [
            ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p, ctypes.c_int, ctypes.c_int,
            ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_float,
            ctypes.c_float, ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
            ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p]
        lib.rnb_bn_seg_apply_f32.argtypes = [
            ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int,
            ctypes.c_int, ctypes.c_void_p, ctypes.c_int, ctypes.c_longlong, ctypes.c_int,
            ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_void_p]
        lib.rnb_bn_seg_apply_f32_ind.argtypes = (lib.rnb_bn_seg_apply_f32.argtypes[:-1]
                                                 + [ctypes.c_void_p, ctypes.c_void_p])
        lib.rnb_bn_seg_apply_sums_f32.argtypes = [
            ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int,
            ctypes.c_int, ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p,
            ctypes.c_float, ctypes.c_int, ctypes.c_longlong, ctypes.c_int, ctypes.c_int,
            ctypes.c_int, ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p]
        lib.rnb_bn_seg_ss_from_sums_f32.argtypes = [
            ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p, ctypes.c_int, ctypes.c_int,
            ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_float, ctypes.c_void_p,
            ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p]
        lib.rnb_bn_seg_set_defer_running.argtypes = [ctypes.c_int]
        lib.rnb_bn_seg_set_defer_running.restype = None
        lib.rnb_bn_seg_defers_running.argtypes = [ctypes.c_int, ctypes.c_int]
        lib.rnb_bn_seg_running_batched.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_int,
                                                   ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p]
        self.bn_run_entry_size = lib.rnb_bn_seg_running_entry_size()
        lib.rnb_bn_seg_walk_apply_f32.argtypes = [
            ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int,
            ctypes.c_int, ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_float,
            ctypes.c_float, ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
            ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
            ctypes.c_int, ctypes.c_longlong, ctypes.c_int, ctypes.c_int, ctypes.c_int,
            ctypes.c_void_p]
        lib.rnb_video_reduce.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                                         ctypes.c_void_p, ctypes.c_int, ctypes.c_int,
                                         ctypes.c_void_p]
        lib.rnb_halo_launch_v.argtypes = [ctypes.POINTER(HaloParams), ctypes.c_int,
                                          ctypes.c_void_p]
        lib.rnb_halo_launch_v.restype = ctypes.c_int
        lib.rnb_halo_lds_bytes_v.argtypes = [ctypes.c_int] * 5
        lib.rnb_temporal_launch.argtypes = [ctypes.POINTER(TemporalParams), ctypes.c_int,
                                            ctypes.c_int, ctypes.c_void_p]
        lib.rnb_temporal_launch.restype = ctypes.c_int
        lib.rnb_temporal_lds_bytes.argtypes = [ctypes.c_int] * 3
        lib.rnb_conv21_launch.argtypes = [ctypes.POINTER(Conv21Params), ctypes.c_void_p]
        lib.rnb_conv21_launch.restype = ctypes.c_int
        lib.rnb_conv21s_launch.argtypes = [ctypes.POINTER(Conv21Params), ctypes.c_void_p]
        lib.rnb_conv21s_launch.restype = ctypes.c_int
        lib.rnb_conv21_supported.argtypes = [ctypes.c_int] * 3
        lib.rnb_conv21_fits.argtypes = [ctypes.c_int] * 6
        if lib.rnb_conv21_params_size() != ctypes.sizeof(Conv21Params):
            raise NativeUnavailable("Conv21Params layout mismatch: rebuild")
        if lib.rnb_temporal_params_size() != ctypes.sizeof(TemporalParams):
            raise NativeUnavailable("TemporalParams layout mismatch: rebuild")
        if lib.rnb_halo_params_size() != ctypes.sizeof(HaloParams):
            raise NativeUnavailable("HaloParams layout mismatch: rebuild")
        if lib.rnb_conv_params_size() != ctypes.sizeof(ConvParams):
            raise NativeUnavailable("ConvParams layout mismatch (%d vs %d): rebuild"
                                    % (lib.rnb_conv_params_size(),
                                       ctypes.sizeof(ConvParams)))
        lib.rnb_conv_f32_launch.argtypes = [ctypes.POINTER(ConvParams), ctypes.c_int,
                                            ctypes.c_void_p]
        lib.rnb_conv_f32_launch.restype = ctypes.c_int
        lib.rnb_conv_f32_config_info.argtypes = [ctypes.c_int, ctypes.POINTER(ctypes.c_int),
                                                 ctypes.POINTER(ctypes.c_int)]
        lib.rnb_conv_f32_max_bytes.restype = ctypes.c_longlong
        lib.rnb_conv_x6_launch.argtypes = [ctypes.POINTER(ConvParams), ctypes.c_int,
                                           ctypes.c_void_p]
        lib.rnb_conv_x6_launch.restype = ctypes.c_int
        lib.rnb_conv_x6_launch_stats.argtypes = [ctypes.POINTER(ConvParams), ctypes.c_int,
                                                 ctypes.c_void_p, ctypes.c_void_p,
                                                 ctypes.c_void_p, ctypes.c_int]
        lib.rnb_conv_x6_launch_stats.restype = ctypes.c_int
        lib.rnb_conv_x6_launch_splitk.argtypes = [ctypes.POINTER(ConvParams), ctypes.c_int,
                                                  ctypes.c_void_p, ctypes.c_void_p,
                                                  ctypes.c_void_p, ctypes.c_int, ctypes.c_int,
                                                  ctypes.c_void_p]
        lib.rnb_conv_x6_launch_splitk.restype = ctypes.c_int
        lib.rnb_conv_x6r_launch.argtypes = [ctypes.POINTER(ConvParams), ctypes.c_int,
                                            ctypes.c_void_p, ctypes.c_void_p,
                                            ctypes.c_void_p, ctypes.c_int]
        lib.rnb_conv_x6r_launch.restype = ctypes.c_int
        lib.rnb_conv_x6_config_info.argtypes = [ctypes.c_int, ctypes.POINTER(ctypes.c_int),
                                                ctypes.POINTER(ctypes.c_int)]
        lib.rnb_conv_h3_launch.argtypes = [ctypes.POINTER(ConvParams), ctypes.c_int,
                                           ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                                           ctypes.c_int, ctypes.c_int, ctypes.c_void_p,
                                           ctypes.c_float, ctypes.c_float, ctypes.c_void_p,
                                           ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int]
        lib.rnb_conv_h3_launch.restype = ctypes.c_int
        lib.rnb_bn_tail_arm.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int,
                                        ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                        ctypes.c_void_p, ctypes.c_void_p, ctypes.c_float,
                                        ctypes.c_void_p]
        lib.rnb_bn_tail_arm.restype = ctypes.c_int
        lib.rnb_bn_tail_disarm.argtypes = []
        lib.rnb_bn_tail_disarm.restype = None
        lib.rnb_bn_tail_taken.argtypes = []
        lib.rnb_bn_tail_taken.restype = ctypes.c_int
        lib.rnb_conv_h3_affine_ok.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_int]
        lib.rnb_conv_h3_affine_ok.restype = ctypes.c_int
        lib.rnb_conv_h3r_launch.argtypes = [ctypes.POINTER(ConvParams), ctypes.c_int,
                                            ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                                            ctypes.c_int, ctypes.c_float, ctypes.c_float,
                                            ctypes.c_void_p, ctypes.c_void_p]
        lib.rnb_conv_h3r_launch.restype = ctypes.c_int
        lib.rnb_conv_h3t_launch.argtypes = lib.rnb_conv_h3r_launch.argtypes
        lib.rnb_conv_h3t_launch.restype = ctypes.c_int
        lib.rnb_conv_h3t_pixels.argtypes = [ctypes.c_int, ctypes.c_int]
        # experiment kernels (build.py --exp; absent from the product build):
        # conv_h3u / conv_h3s report 0 variants without their library
        self.exp = None
        exp_path = os.path.join(NATIVE_DIR, "exp", "librnb_h3exp.so")
        if os.path.exists(exp_path) and os.environ.get("RNB_EXP_KERNELS", "1") != "0":
            try:
                self.exp = ctypes.CDLL(exp_path)
            except OSError:
                self.exp = None
        if self.exp is not None:
            ex = self.exp
            ex.rnb_conv_h3u_launch.argtypes = lib.rnb_conv_h3r_launch.argtypes
            ex.rnb_conv_h3u_launch.restype = ctypes.c_int
            ex.rnb_conv_h3u_pixels.argtypes = [ctypes.c_int, ctypes.c_int]
            ex.rnb_conv_h3u_pixels.restype = ctypes.c_int
            ex.rnb_conv_h3s_launch.argtypes = [ctypes.POINTER(ConvParams), ctypes.c_int,
                                               ctypes.c_void_p, ctypes.c_void_p,
                                               ctypes.c_void_p, ctypes.c_int, ctypes.c_float,
                                               ctypes.c_float]
            ex.rnb_conv_h3s_launch.restype = ctypes.c_int
            ex.rnb_conv_h3s_rows.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_int]
            ex.rnb_conv_h3s_rows.restype = ctypes.c_int
        lib.rnb_conv_h3stem_launch.argtypes = [ctypes.POINTER(ConvParams), ctypes.c_int,
                                               ctypes.c_void_p, ctypes.c_void_p,
                                               ctypes.c_void_p, ctypes.c_int, ctypes.c_float,
                                               ctypes.c_float]
        lib.rnb_conv_h3stem_launch.restype = ctypes.c_int
        lib.rnb_conv_h3stem_rows.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_int]
        lib.rnb_conv_h3stem_rows.restype = ctypes.c_int
        lib.rnb_conv_h3p_launch.argtypes = [ctypes.POINTER(ConvParams), ctypes.c_int,
                                            ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                                            ctypes.c_int, ctypes.c_float, ctypes.c_float,
                                            ctypes.c_void_p, ctypes.c_void_p]
        lib.rnb_conv_h3p_launch.restype = ctypes.c_int
        lib.rnb_conv_h3p_ok.argtypes = [ctypes.c_int] * 5
        lib.rnb_conv_h3p_ok.restype = ctypes.c_int
        lib.rnb_conv_h3w_launch.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p,
                                            ctypes.c_float, ctypes.c_float, ctypes.c_void_p]
        lib.rnb_conv_h3w_launch.restype = ctypes.c_int
        lib.rnb_conv_h3w_tc.argtypes = [ctypes.c_int]
        lib.rnb_conv_h3w_tc.restype = ctypes.c_int
        lib.rnb_h3_set_range_flag.argtypes = [ctypes.c_void_p]
        lib.rnb_h3_set_range_flag.restype = None
        lib.rnb_conv_h3t_pixels.restype = ctypes.c_int
        lib.rnb_conv_h3_config_info.argtypes = [ctypes.c_int, ctypes.POINTER(ctypes.c_int),
                                                ctypes.POINTER(ctypes.c_int)]
        lib.rnb_preprocess_f32.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_longlong,
                                           ctypes.POINTER(ctypes.c_float),
                                           ctypes.POINTER(ctypes.c_float), ctypes.c_void_p]
        lib.rnb_head_f32.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                                     ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int,
                                     ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                     ctypes.c_void_p]
        lib.rnb_wino_f32_launch.argtypes = [ctypes.POINTER(WinoParams), ctypes.c_int,
                                            ctypes.c_void_p]
        lib.rnb_wino_f32_launch.restype = ctypes.c_int
        lib.rnb_winot_f32_launch.argtypes = [ctypes.POINTER(WinoParams), ctypes.c_int,
                                             ctypes.c_void_p]
        lib.rnb_winot_f32_launch.restype = ctypes.c_int
        for fn in (lib.rnb_wino_x6_launch, lib.rnb_winot_x6_launch):
            fn.argtypes = [ctypes.POINTER(WinoParams), ctypes.c_int, ctypes.c_void_p]
            fn.restype = ctypes.c_int
        if lib.rnb_wino_params_size() != ctypes.sizeof(WinoParams):
            raise NativeUnavailable("WinoParams layout mismatch: rebuild")
        if lib.rnb_conv_f32_params_size() != ctypes.sizeof(ConvParams):
            raise NativeUnavailable("ConvF32Params layout mismatch: rebuild")
        self.f32_configs = []      # (pixel tile, channel tile) per fp32 config id
        for i in range(lib.rnb_conv_f32_num_configs()):
            p, c = ctypes.c_int(), ctypes.c_int()
            lib.rnb_conv_f32_config_info(i, ctypes.byref(p), ctypes.byref(c))
            self.f32_configs.append((p.value, c.value))
        self.f32_max_bytes = lib.rnb_conv_f32_max_bytes()
        self.x6r_variants = lib.rnb_conv_x6r_num_variants()
        self.h3r_variants = lib.rnb_conv_h3r_num_variants()
        self.h3t_variants = lib.rnb_conv_h3t_num_variants()
        self.h3w_variants = lib.rnb_conv_h3w_num_variants()
        self.h3u_variants = self.exp.rnb_conv_h3u_num_variants() if self.exp else 0
        self.h3s_variants = self.exp.rnb_conv_h3s_num_variants() if self.exp else 0
        self.h3stem_variants = lib.rnb_conv_h3stem_num_variants()
        self.x6_configs = []       # (pixel tile, channel tile) per x6 direct config
        for i in range(lib.rnb_conv_x6_num_configs()):
            p, c = ctypes.c_int(), ctypes.c_int()
            lib.rnb_conv_x6_config_info(i, ctypes.byref(p), ctypes.byref(c))
            self.x6_configs.append((p.value, c.value))
        self.h3_configs = []       # (pixel tile, channel tile) per h3 direct config
        for i in range(lib.rnb_conv_h3_num_configs()):
            p, c = ctypes.c_int(), ctypes.c_int()
            lib.rnb_conv_h3_config_info(i, ctypes.byref(p), ctypes.byref(c))
            self.h3_configs.append((p.value, c.value))
        self.configs = []          # (pixel tile, channel tile) per config id
        self.stages = []           # LDS staging depth per config id
        for i in range(lib.rnb_conv_num_configs()):
            p, c = ctypes.c_int(), ctypes.c_int()
            lib.rnb_conv_config_info(i, ctypes.byref(p), ctypes.byref(c))
            self.configs.append((p.value, c.value))
            self.stages.append(lib.rnb_conv_config_stages(i))

    def conv(self, params: ConvParams, config_id: int, stream: int) -> None:
        _check(self.lib.rnb_conv_launch(ctypes.byref(params), config_id, stream),
               "conv (config %d)" % config_id)

    def conv_f32(self, params: ConvParams, config_id: int, stream: int) -> None:
        _check(self.lib.rnb_conv_f32_launch(ctypes.byref(params), config_id, stream),
               "conv_f32 (config %d)" % config_id)

    def conv_x6(self, params: ConvParams, config_id: int, stream: int, sums: int = 0,
                clip_seg: int = 0, stats_c: int = 0, ksplit: int = 1, ws: int = 0) -> None:
        """x6 direct conv; ``sums`` (fp64 [nseg][2][stats_c] device pointer, with
        ``clip_seg`` int32 [N]): add the output's per-video BN sums. ``ksplit`` >
        1: split-K over that many blocks per tile with ``ws`` (fp32, ksplit x M x
        Cout_p) for the partials, finished by a reduce kernel."""
        _check(self.lib.rnb_conv_x6_launch_splitk(ctypes.byref(params), config_id, stream,
                                                  sums or None, clip_seg or None, stats_c,
                                                  ksplit, ws or None),
               "conv_x6 (config %d, ksplit %d)" % (config_id, ksplit))

    def conv_h3(self, params: ConvParams, config_id: int, stream: int, in_scale: float,
                out_scale: float, sums: int = 0, clip_seg: int = 0, stats_c: int = 0,
                ksplit: int = 1, ws: int = 0, in_ss: int = 0, in_seg: int = 0,
                tick: int = 0, tick_cap: int = 0) -> None:
        """h3 direct conv (fp32 products as fp16 hi/lo products, csrc/conv_h3.hip):
        ``params.w`` = split weights scaled by 2^sw, ``in_scale`` = 2^sa applied
        to the activations, ``out_scale`` = 2^-(sa + sw); sums / ksplit / ws as
        ``conv_x6``; ``in_ss`` (fp32 [nseg][2][Cin_p] scale/shift) with
        ``in_seg`` (int32 [N] video per clip): the input's BatchNorm + ReLU
        applied on load. ``tick`` (split-K): int32 [>= tiles] zeroed arrival
        counters (``tick_cap`` entries): the last block of each tile finishes
        it in the same dispatch instead of a reduce kernel."""
        _check(self.lib.rnb_conv_h3_launch(ctypes.byref(params), config_id, stream,
                                           sums or None, clip_seg or None, stats_c, ksplit,
                                           ws or None, in_scale, out_scale, in_ss or None,
                                           in_seg or None, tick or None, tick_cap),
               "conv_h3 (config %d, ksplit %d)" % (config_id, ksplit))

    def bn_tail_arm(self, ticket, sums, sums_c, coffs, nseg, rpc, C, gamma, beta, eps,
                    ss) -> None:
        """Arms the BN finalize (scale / shift rows into ``ss``) for the next
        conv launch that supports it (csrc/bn_tail.h); see ``bn_tail_taken``."""
        _check(self.lib.rnb_bn_tail_arm(ticket, sums, sums_c, coffs, nseg, rpc, C, gamma, beta,
                                        eps, ss), "bn_tail_arm")

    def bn_aff_arm(self, sums, sums_c, coffs, nseg, rpc, C, gamma, beta, eps, ss) -> None:
        """The next h3 direct launches whose input BN rows are ``ss`` compute
        them from the producer's fp64 ``sums`` (csrc/bn_tail.h BnAffSums)."""
        _check(self.lib.rnb_bn_aff_arm(sums, sums_c, coffs, nseg, rpc, C, gamma, beta, eps, ss),
               "bn_aff_arm")

    def bn_aff_disarm(self) -> None:
        self.lib.rnb_bn_aff_disarm()

    def bn_aff_used(self) -> bool:
        """True when a launch computed the armed rows since the last call."""
        return bool(self.lib.rnb_bn_aff_used())

    def bn_set_apply_blk(self, on: bool) -> None:
        """Block-tiled BN applies (bn_seg_apply_blk_f32_kernel) on / off."""
        self.lib.rnb_bn_set_apply_blk(1 if on else 0)

    def bn_tail_disarm(self) -> None:
        self.lib.rnb_bn_tail_disarm()

    def bn_tail_taken(self) -> bool:
        """True when a launch took the last armed BN tail (resets)."""
        return bool(self.lib.rnb_bn_tail_taken())

    def h3_set_range_flag(self, dev_ptr: int) -> None:
        """Range-guard flag (device address of host-coherent memory, 0 = none)
        written by the h3 launches that follow when an output is non-finite."""
        self.lib.rnb_h3_set_range_flag(dev_ptr or None)

    def conv_h3r(self, params: ConvParams, variant: int, stream: int, in_scale: float,
                 out_scale: float, sums: int = 0, clip_seg: int = 0, stats_c: int = 0,
                 in_ss: int = 0, in_seg: int = 0) -> None:
        """h3 row-band halo conv (1x3x3 stride 1 pad 1, Cin_p % 32 == 0); the
        arguments as ``conv_h3``."""
        _check(self.lib.rnb_conv_h3r_launch(ctypes.byref(params), variant, stream,
                                            sums or None, clip_seg or None, stats_c, in_scale,
                                            out_scale, in_ss or None, in_seg or None),
               "conv_h3r (variant %d)" % variant)

    def conv_h3t(self, params: ConvParams, variant: int, stream: int, in_scale: float,
                 out_scale: float, sums: int = 0, clip_seg: int = 0, stats_c: int = 0,
                 in_ss: int = 0, in_seg: int = 0) -> None:
        """h3 temporal frame-band conv (3x1x1 stride 1 pad (1, 0, 0), weights
        padded per tap to 32-channel chunks); the arguments as ``conv_h3``."""
        _check(self.lib.rnb_conv_h3t_launch(ctypes.byref(params), variant, stream,
                                            sums or None, clip_seg or None, stats_c, in_scale,
                                            out_scale, in_ss or None, in_seg or None),
               "conv_h3t (variant %d)" % variant)

    def conv_h3u(self, params: ConvParams, variant: int, stream: int, in_scale: float,
                 out_scale: float, sums: int = 0, clip_seg: int = 0, stats_c: int = 0,
                 in_ss: int = 0, in_seg: int = 0) -> None:
        """Wave-specialised temporal h3 conv (csrc/conv_h3u.hip: staging waves
        split the next chunk while the MFMA waves run the current one); the
        weights and arguments as ``conv_h3t``."""
        _check(self.exp.rnb_conv_h3u_launch(ctypes.byref(params), variant, stream,
                                            sums or None, clip_seg or None, stats_c, in_scale,
                                            out_scale, in_ss or None, in_seg or None),
               "conv_h3u (variant %d)" % variant)

    def conv_h3s(self, params: ConvParams, variant: int, stream: int, in_scale: float,
                 out_scale: float, sums: int = 0, clip_seg: int = 0, stats_c: int = 0) -> None:
        """h3 stride-2 row-band halo conv (csrc/conv_h3s.hip: 1x3x3 stride
        (1, 2, 2) pad (0, 1, 1), Cin_p % 32 == 0, the h3 direct weights); the
        arguments as ``conv_h3`` (no input BN on load)."""
        _check(self.exp.rnb_conv_h3s_launch(ctypes.byref(params), variant, stream,
                                            sums or None, clip_seg or None, stats_c, in_scale,
                                            out_scale),
               "conv_h3s (variant %d)" % variant)

    def conv_h3stem(self, params: ConvParams, variant: int, stream: int, in_scale: float,
                    out_scale: float, sums: int = 0, clip_seg: int = 0, stats_c: int = 0) -> None:
        """h3 stem conv (csrc/conv_h3stem.hip: 1x7x7 stride (1, 2, 2) pad (0, 3, 3),
        Cin_p 4, K-permuted weights -- ConvLayerF32.h3stem_buffers); the
        arguments as ``conv_h3s``."""
        _check(self.lib.rnb_conv_h3stem_launch(ctypes.byref(params), variant, stream,
                                               sums or None, clip_seg or None, stats_c, in_scale,
                                               out_scale),
               "conv_h3stem (variant %d)" % variant)

    def conv_h3p(self, params: ConvParams, blocks_per_cu: int, stream: int, in_scale: float,
                 out_scale: float, sums: int = 0, clip_seg: int = 0, stats_c: int = 0,
                 in_ss: int = 0, in_seg: int = 0) -> None:
        """Pixel-major persistent temporal h3 conv (csrc/conv_h3p.hip: 3x1x1
        stride 1 pad (1, 0, 0), T 8, Cin_p <= 160, Cout_p <= 64, all weights
        in LDS; ``blocks_per_cu`` persistent blocks per CU); the weights and
        the other arguments as ``conv_h3t``."""
        _check(self.lib.rnb_conv_h3p_launch(ctypes.byref(params), blocks_per_cu, stream,
                                            sums or None, clip_seg or None, stats_c, in_scale,
                                            out_scale, in_ss or None, in_seg or None),
               "conv_h3p (%d blocks per CU)" % blocks_per_cu)

    def conv_h3w(self, params: "WinoParams", variant: int, stream: int, in_scale: float,
                 out_scale: float, out_seg: int = 0) -> None:
        """Winograd F(2x2, 3x3) h3 conv (csrc/conv_h3w.hip: 1x3x3 stride 1 pad 1,
        Cin_p % 16 == 0, U split into fp16 hi / lo on the host --
        ConvLayerF32.h3w_u); input BN on load when ``params.in_ss`` is set,
        epilogue BN sums when ``params.out_stats`` is set (videos of the clips in
        ``out_seg``; ``params.clip_seg``: the input BN's)."""
        _check(self.lib.rnb_conv_h3w_launch(ctypes.byref(params), variant, stream, in_scale,
                                            out_scale, out_seg or None),
               "conv_h3w (variant %d)" % variant)

    def conv_h3w_tc(self, variant: int) -> int:
        """16-channel groups per work unit of h3w variant ``variant``."""
        return int(self.lib.rnb_conv_h3w_tc(variant))

    def conv_h3p_ok(self, T: int, H: int, W: int, Cin_p: int, Cout_p: int) -> bool:
        return bool(self.lib.rnb_conv_h3p_ok(T, H, W, Cin_p, Cout_p))

    def conv_h3stem_rows(self, variant: int, Ho: int, Wo: int) -> int:
        return int(self.lib.rnb_conv_h3stem_rows(variant, Ho, Wo))

    def conv_h3s_rows(self, variant: int, Ho: int, Wo: int) -> int:
        """Output rows per band of h3s variant ``variant`` (0: cannot run)."""
        return int(self.exp.rnb_conv_h3s_rows(variant, Ho, Wo)) if self.exp else 0

    def conv_h3u_pixels(self, variant: int, T: int) -> int:
        return int(self.exp.rnb_conv_h3u_pixels(variant, T)) if self.exp else 0

    def conv_h3t_pixels(self, variant: int, T: int) -> int:
        """Pixels per block of h3t variant ``variant`` for T frames (0: cannot run)."""
        return int(self.lib.rnb_conv_h3t_pixels(variant, T))

    def conv_h3_affine_ok(self, config_id: int, cin_p: int, rows_per_clip: int) -> bool:
        return bool(self.lib.rnb_conv_h3_affine_ok(config_id, cin_p, rows_per_clip))

    def conv_x6r(self, params: ConvParams, variant: int, stream: int, sums: int = 0,
                 clip_seg: int = 0, stats_c: int = 0) -> None:
        """x6 row-band halo conv (1x3x3 stride 1 pad 1), optional BN sums."""
        _check(self.lib.rnb_conv_x6r_launch(ctypes.byref(params), variant, stream,
                                            sums or None, clip_seg or None, stats_c),
               "conv_x6r (variant %d)" % variant)

    def wino_f32(self, params: "WinoParams", variant: int, stream: int) -> None:
        _check(self.lib.rnb_wino_f32_launch(ctypes.byref(params), variant, stream),
               "conv_wino_f32 (variant %d)" % variant)

    def winot_f32(self, params: "WinoParams", variant: int, stream: int) -> None:
        _check(self.lib.rnb_winot_f32_launch(ctypes.byref(params), variant, stream),
               "conv_winot_f32 (variant %d)" % variant)

    def wino_x6(self, params: "WinoParams", variant: int, stream: int) -> None:
        _check(self.lib.rnb_wino_x6_launch(ctypes.byref(params), variant, stream),
               "conv_wino_x6 (variant %d)" % variant)

    def winot_x6(self, params: "WinoParams", variant: int, stream: int) -> None:
        _check(self.lib.rnb_winot_x6_launch(ctypes.byref(params), variant, stream),
               "conv_winot_x6 (variant %d)" % variant)

    def preprocess_f32(self, in_ptr, out_ptr, npix, mean, std, stream):
        m = (ctypes.c_float * 3)(*mean)
        s = (ctypes.c_float * 3)(*std)
        _check(self.lib.rnb_preprocess_f32(in_ptr, out_ptr, npix, m, s, stream),
               "preprocess_f32")

    def head_f32(self, x_ptr, w_ptr, b_ptr, out_ptr, pooled_ptr, N, S, C, Cs, ncls, stream):
        _check(self.lib.rnb_head_f32(x_ptr, w_ptr, b_ptr, out_ptr, pooled_ptr, N, S, C, Cs,
                                     ncls, stream), "head_f32")

    def halo(self, params: HaloParams, stream: int, variant: int = 2) -> None:
        """variant (csrc/conv_halo.hip kHalo): 2 = 32-pixel waves, 4 = 64-pixel
        waves, 5 = 64-pixel waves over 448-pixel tiles."""
        _check(self.lib.rnb_halo_launch_v(ctypes.byref(params), variant, stream), "conv_halo")

    def temporal(self, params: TemporalParams, num_cus: int, blocks_per_cu: int,
                 stream: int) -> None:
        _check(self.lib.rnb_temporal_launch(ctypes.byref(params), num_cus, blocks_per_cu,
                                            stream), "conv_temporal")

    def conv21(self, params: Conv21Params, stream: int, variant: int = 1) -> None:
        """Fused spatial 1x3x3 (64 -> 144) + temporal 3x1x1 (144 -> 64).
        variant 1: role-specialised 8-wave kernel (conv21s), 0: 4-wave kernel."""
        fn = self.lib.rnb_conv21s_launch if variant == 1 else self.lib.rnb_conv21_launch
        _check(fn(ctypes.byref(params), stream), "conv21 (variant %d)" % variant)

    def conv21_supported(self, T: int, H: int, W: int) -> bool:
        return bool(self.lib.rnb_conv21_supported(T, H, W))

    def conv21_fits(self, N: int, T: int, H: int, W: int, y_stride: int = 64,
                    res_stride: int = 64) -> bool:
        """Whole launch contract for N clips (buffer-offset limits included)."""
        return bool(self.lib.rnb_conv21_fits(N, T, H, W, y_stride, res_stride))

    def temporal_lds_bytes(self, T: int, cin_p: int, cout_p: int) -> int:
        return self.lib.rnb_temporal_lds_bytes(T, cin_p, cout_p)

    def halo_lds_bytes(self, frames: int, H: int, W: int, cin: int, variant: int = 2) -> int:
        return self.lib.rnb_halo_lds_bytes_v(frames, H, W, cin, variant)

    def bn_scratch_floats(self, M: int, C: int) -> int:
        return self.lib.rnb_bn_scratch_floats(M, C)

    def bn_stats(self, y_ptr, M, C, stride, scratch_ptr, mean_ptr, var_ptr, stream):
        _check(self.lib.rnb_bn_stats(y_ptr, M, C, stride, scratch_ptr, mean_ptr, var_ptr,
                                     stream), "bn_stats")

    def bn_apply(self, y_ptr, z_ptr, res_ptr, mean_ptr, var_ptr, gamma_ptr, beta_ptr, eps,
                 relu, M, C, y_stride, z_stride, res_stride, stream):
        _check(self.lib.rnb_bn_apply(y_ptr, z_ptr, res_ptr, mean_ptr, var_ptr, gamma_ptr,
                                     beta_ptr, eps, relu, M, C, y_stride, z_stride, res_stride,
                                     stream), "bn_apply")

    def bn_seg_bps(self, nseg: int, C: int, M: int) -> int:
        return self.lib.rnb_bn_seg_bps(nseg, C, M)

    def bn_seg_scratch_floats(self, nseg: int, C: int, M: int) -> int:
        return self.lib.rnb_bn_seg_scratch_floats(nseg, C, M)

    def bn_seg_stats_f32(self, y_ptr, coffs_ptr, nseg, rpc, M, C, stride, scratch_ptr,
                         scratch_floats, run_acc_ptr, gamma_ptr, beta_ptr, eps, momentum,
                         channels, rmean_ptr, rvar_ptr, mean_ptr, var_ptr, ss_ptr, stream):
        _check(self.lib.rnb_bn_seg_stats_f32(y_ptr, coffs_ptr, nseg, rpc, M, C, stride,
                                             scratch_ptr, scratch_floats, run_acc_ptr, gamma_ptr, beta_ptr, eps, momentum,
                                             channels, rmean_ptr, rvar_ptr, mean_ptr, var_ptr,
                                             ss_ptr, stream), "bn_seg_stats_f32")

    def bn_seg_stats_from_sums_f32(self, sums_ptr, sums_c, coffs_ptr, nseg, rpc, C, run_acc_ptr,
                                   gamma_ptr, beta_ptr, eps, momentum, channels, rmean_ptr,
                                   rvar_ptr, mean_ptr, var_ptr, ss_ptr, stream):
        _check(self.lib.rnb_bn_seg_stats_from_sums_f32(
            sums_ptr, sums_c, coffs_ptr, nseg, rpc, C, run_acc_ptr, gamma_ptr, beta_ptr, eps,
            momentum, channels, rmean_ptr, rvar_ptr, mean_ptr, var_ptr, ss_ptr, stream),
            "bn_seg_stats_from_sums_f32")

    def bn_seg_set_defer_running(self, on: bool) -> None:
        """Finalize paths that would launch a separate running-update kernel
        leave it to the caller (``bn_seg_running_batched``) while on."""
        self.lib.rnb_bn_seg_set_defer_running(1 if on else 0)

    def bn_seg_defers_running(self, nseg: int, from_sums: bool) -> bool:
        return bool(self.lib.rnb_bn_seg_defers_running(nseg, 1 if from_sums else 0))

    def bn_seg_running_batched(self, table_ptr, n, max_channels, coffs_ptr, nseg, stream):
        _check(self.lib.rnb_bn_seg_running_batched(table_ptr, n, max_channels, coffs_ptr, nseg,
                                                   stream), "bn_seg_running_batched")

    def bn_seg_apply_f32(self, y_ptr, z_ptr, res_ptr, coffs_ptr, nseg, rpc, ss_ptr, relu, M, C,
                         y_stride, z_stride, res_stride, stream, zind_ptr=None):
        """``zind_ptr``: device address of an 8-byte pointer the kernel reads
        as its destination instead of ``z_ptr`` (graphs writing into a slot)."""
        _check(self.lib.rnb_bn_seg_apply_f32_ind(y_ptr, z_ptr, res_ptr, coffs_ptr, nseg, rpc,
                                                 ss_ptr, relu, M, C, y_stride, z_stride,
                                                 res_stride, zind_ptr or None, stream),
               "bn_seg_apply_f32")

    def bn_seg_ss_from_sums_f32(self, sums_ptr, sums_c, coffs_ptr, nseg, rpc, C, gamma_ptr,
                                beta_ptr, eps, mean_ptr, var_ptr, ss_ptr, stream):
        """Scale / shift (+ moments) from epilogue sums, no running update and
        no re-arm (the batched running update does both)."""
        _check(self.lib.rnb_bn_seg_ss_from_sums_f32(sums_ptr, sums_c, coffs_ptr, nseg, rpc, C,
                                                    gamma_ptr, beta_ptr, eps, mean_ptr, var_ptr,
                                                    ss_ptr, stream), "bn_seg_ss_from_sums_f32")

    def bn_seg_apply_sums_f32(self, y_ptr, z_ptr, res_ptr, coffs_ptr, nseg, rpc, sums_ptr,
                              sums_c, gamma_ptr, beta_ptr, eps, relu, M, C, y_stride, z_stride,
                              res_stride, stream, zind_ptr=None):
        """The apply with its scale / shift computed from the producer
        epilogue's fp64 sums (no finalize kernel); the sums are left for the
        batched running update to walk and re-arm."""
        _check(self.lib.rnb_bn_seg_apply_sums_f32(y_ptr, z_ptr, res_ptr, coffs_ptr, nseg, rpc,
                                                  sums_ptr, sums_c, gamma_ptr, beta_ptr, eps,
                                                  relu, M, C, y_stride, z_stride, res_stride,
                                                  zind_ptr or None, stream),
               "bn_seg_apply_sums_f32")

    def bn_seg_walk_apply_f32(self, sums_ptr, sums_c, ticket_ptr, coffs_ptr, nseg, rpc, C,
                              gamma_ptr, beta_ptr, eps, momentum, channels, rmean_ptr, rvar_ptr,
                              mean_ptr, var_ptr, ss_ptr, y_ptr, z_ptr, res_ptr, relu, M,
                              y_stride, z_stride, res_stride, stream):
        _check(self.lib.rnb_bn_seg_walk_apply_f32(
            sums_ptr, sums_c, ticket_ptr, coffs_ptr, nseg, rpc, C, gamma_ptr, beta_ptr, eps,
            momentum, channels, rmean_ptr, rvar_ptr, mean_ptr, var_ptr, ss_ptr, y_ptr, z_ptr,
            res_ptr, relu, M, y_stride, z_stride, res_stride, stream), "bn_seg_walk_apply_f32")

    def clipgen_u8(self, out_ptr, vids_ptr, starts_ptr, nclips, F, H, W, stream):
        _check(self.lib.rnb_clipgen_u8(out_ptr, vids_ptr, starts_ptr, nclips, F, H, W,
                                       stream), "clipgen_u8")

    def clipgen_video(self, out_ptr, vid, starts, F, H, W, stream):
        arr = (ctypes.c_int * max(1, len(starts)))(*starts)
        _check(self.lib.rnb_clipgen_video(out_ptr, int(vid), arr, len(starts), F, H, W,
                                          stream), "clipgen_video")

    def nv12gen_video(self, out_ptr, vid, starts, F, H, W, stream):
        arr = (ctypes.c_int * max(1, len(starts)))(*starts)
        _check(self.lib.rnb_nv12gen_video(out_ptr, int(vid), arr, len(starts), F, H, W,
                                          stream), "nv12gen_video")

    def nv12gen(self, out_ptr, vids_ptr, starts_ptr, nclips, F, H, W, stream):
        _check(self.lib.rnb_nv12gen(out_ptr, vids_ptr, starts_ptr, nclips, F, H, W, stream),
               "nv12gen")

    def nv12_to_clip(self, in_ptr, out_ptr, frames, src_w, src_h, out_w, out_h, crop, mean,
                     std, bf16, stream):
        c = (ctypes.c_float * 4)(*crop)
        m = (ctypes.c_float * 3)(*mean)
        s = (ctypes.c_float * 3)(*std)
        _check(self.lib.rnb_nv12_to_clip(in_ptr, out_ptr, frames, src_w, src_h, out_w, out_h,
                                         c, m, s, 1 if bf16 else 0, stream), "nv12_to_clip")

    def preprocess(self, in_ptr, out_ptr, npix, mean, std, stream):
        m = (ctypes.c_float * 3)(*mean)
        s = (ctypes.c_float * 3)(*std)
        _check(self.lib.rnb_preprocess(in_ptr, out_ptr, npix, m, s, stream), "preprocess")

    def stem_pack(self, in_ptr, out_ptr, frames, H, W, stream):
        _check(self.lib.rnb_stem_pack(in_ptr, out_ptr, frames, H, W, stream), "stem_pack")

    def preprocess_packed(self, in_ptr, out_ptr, frames, H, W, mean, std, stream):
        m = (ctypes.c_float * 3)(*mean)
        s = (ctypes.c_float * 3)(*std)
        _check(self.lib.rnb_preprocess_packed(in_ptr, out_ptr, frames, H, W, m, s, stream),
               "preprocess_packed")

    def head(self, x_ptr, w_ptr, b_ptr, out_ptr, pooled_ptr, N, S, C, Cs, ncls, stream):
        _check(self.lib.rnb_head(x_ptr, w_ptr, b_ptr, out_ptr, pooled_ptr, N, S, C, Cs, ncls,
                                 stream), "head")

    def video_reduce(self, logits_ptr, offsets_ptr, sums_ptr, argmax_ptr, nvid, ncls,
                     stream):
        _check(self.lib.rnb_video_reduce(logits_ptr, offsets_ptr, sums_ptr, argmax_ptr,
                                         nvid, ncls, stream), "video_reduce")


class Runtime:
    """Typed wrappers over librnb_runtime.so (IPC, copies, device info)."""

    def __init__(self):
        lib = _load("librnb_runtime.so")
        self.lib = lib
        vp, sz = ctypes.c_void_p, ctypes.c_size_t
        lib.rnb_error_string.restype = ctypes.c_char_p
        lib.rnb_malloc.argtypes = [ctypes.POINTER(vp), sz]
        lib.rnb_free.argtypes = [vp]
        lib.rnb_host_alloc_mapped.argtypes = [sz, ctypes.POINTER(vp), ctypes.POINTER(vp)]
        lib.rnb_host_free.argtypes = [vp]
        lib.rnb_ipc_get_mem_handle.argtypes = [vp, vp]
        lib.rnb_ipc_open_mem_handle.argtypes = [vp, ctypes.POINTER(vp)]
        lib.rnb_ipc_close_mem_handle.argtypes = [vp]
        lib.rnb_memcpy_async.argtypes = [vp, vp, sz, vp]
        lib.rnb_memcpy_d2h.argtypes = [vp, vp, sz]
        lib.rnb_memcpy_peer_async.argtypes = [vp, ctypes.c_int, vp, ctypes.c_int, sz, vp]
        lib.rnb_stream_synchronize.argtypes = [vp]
        lib.rnb_ipc_event_create.argtypes = [ctypes.POINTER(vp)]
        lib.rnb_ipc_get_event_handle.argtypes = [vp, vp]
        lib.rnb_ipc_open_event_handle.argtypes = [vp, ctypes.POINTER(vp)]
        lib.rnb_event_record.argtypes = [vp, vp]
        lib.rnb_stream_wait_event.argtypes = [vp, vp]
        lib.rnb_event_synchronize.argtypes = [vp]
        lib.rnb_event_query.argtypes = [vp]
        lib.rnb_clear_last_error.argtypes = []
        lib.rnb_event_destroy.argtypes = [vp]
        lib.rnb_can_access_peer.argtypes = [ctypes.c_int, ctypes.c_int,
                                            ctypes.POINTER(ctypes.c_int)]
        lib.rnb_mem_get_info.argtypes = [ctypes.POINTER(sz), ctypes.POINTER(sz)]
        lib.rnb_stream_create.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.POINTER(vp)]
        lib.rnb_stream_destroy.argtypes = [vp]
        lib.rnb_stream_create_cumask.argtypes = [ctypes.POINTER(ctypes.c_uint32), ctypes.c_int,
                                                 ctypes.POINTER(vp)]
        lib.rnb_spin.argtypes = [vp, ctypes.c_longlong]
        self.handle_size = lib.rnb_ipc_handle_size()
        self.event_handle_size = lib.rnb_ipc_event_handle_size()

    def set_device(self, dev: int) -> None:
        _check(self.lib.rnb_set_device(dev), "hipSetDevice")

    def stream_create(self, nonblocking: bool = True, priority: int = 0) -> int:
        s = ctypes.c_void_p()
        _check(self.lib.rnb_stream_create(int(nonblocking), priority, ctypes.byref(s)),
               "hipStreamCreateWithPriority")
        return s.value

    def stream_create_cumask(self, enabled_cus) -> int:
        """A stream limited to the CUs in ``enabled_cus`` (indices) of the
        current device (hipExtStreamCreateWithCUMask)."""
        cus = sorted(set(int(c) for c in enabled_cus))
        n = (max(cus) // 32 + 1) if cus else 1
        words = (ctypes.c_uint32 * n)()
        for c in cus:
            words[c // 32] |= 1 << (c % 32)
        s = ctypes.c_void_p()
        _check(self.lib.rnb_stream_create_cumask(words, n, ctypes.byref(s)),
               "hipExtStreamCreateWithCUMask")
        return s.value

    def stream_destroy(self, stream: int) -> None:
        _check(self.lib.rnb_stream_destroy(stream), "hipStreamDestroy")

    def spin(self, stream: int, cycles: int) -> None:
        """Busy-wait kernel of ~``cycles`` GPU clocks on ``stream``."""
        _check(self.lib.rnb_spin(stream, cycles), "spin kernel")

    def ipc_malloc(self, nbytes: int) -> int:
        p = ctypes.c_void_p()
        _check(self.lib.rnb_malloc(ctypes.byref(p), nbytes), "hipMalloc(%d)" % nbytes)
        return p.value

    def free(self, ptr: int) -> None:
        _check(self.lib.rnb_free(ptr), "hipFree")

    def host_alloc_mapped(self, nbytes: int):
        """(host pointer, device pointer) of zeroed host-coherent memory the
        GPU can write (hipHostMalloc mapped | coherent)."""
        h, d = ctypes.c_void_p(), ctypes.c_void_p()
        _check(self.lib.rnb_host_alloc_mapped(nbytes, ctypes.byref(h), ctypes.byref(d)),
               "hipHostMalloc(%d)" % nbytes)
        return h.value, d.value

    def host_free(self, host: int) -> None:
        _check(self.lib.rnb_host_free(host), "hipHostFree")

    def ipc_get_handle(self, ptr: int) -> bytes:
        buf = ctypes.create_string_buffer(self.handle_size)
        _check(self.lib.rnb_ipc_get_mem_handle(ptr, buf), "hipIpcGetMemHandle")
        return buf.raw

    def ipc_open_handle(self, handle: bytes) -> int:
        p = ctypes.c_void_p()
        buf = ctypes.create_string_buffer(handle, len(handle))
        _check(self.lib.rnb_ipc_open_mem_handle(buf, ctypes.byref(p)),
               "hipIpcOpenMemHandle")
        return p.value

    def ipc_close_handle(self, ptr: int) -> None:
        _check(self.lib.rnb_ipc_close_mem_handle(ptr), "hipIpcCloseMemHandle")

    def event_create_ipc(self) -> int:
        p = ctypes.c_void_p()
        _check(self.lib.rnb_ipc_event_create(ctypes.byref(p)), "hipEventCreate")
        return p.value

    def event_get_handle(self, ev: int) -> bytes:
        buf = ctypes.create_string_buffer(self.event_handle_size)
        _check(self.lib.rnb_ipc_get_event_handle(ev, buf), "hipIpcGetEventHandle")
        return buf.raw

    def event_open_handle(self, handle: bytes) -> int:
        p = ctypes.c_void_p()
        buf = ctypes.create_string_buffer(handle, len(handle))
        _check(self.lib.rnb_ipc_open_event_handle(buf, ctypes.byref(p)),
               "hipIpcOpenEventHandle")
        return p.value

    def event_record(self, ev: int, stream: int) -> None:
        _check(self.lib.rnb_event_record(ev, stream), "hipEventRecord")

    def stream_wait_event(self, stream: int, ev: int) -> None:
        _check(self.lib.rnb_stream_wait_event(stream, ev), "hipStreamWaitEvent")

    def try_stream_wait_event(self, stream: int, ev: int) -> int:
        """hipStreamWaitEvent's error code (0 = ok) instead of raising."""
        return int(self.lib.rnb_stream_wait_event(stream, ev))

    def event_synchronize(self, ev: int) -> None:
        _check(self.lib.rnb_event_synchronize(ev), "hipEventSynchronize")

    def clear_last_error(self) -> int:
        return int(self.lib.rnb_clear_last_error())

    def event_query(self, ev: int) -> int:
        return int(self.lib.rnb_event_query(ev))

    def event_destroy(self, ev: int) -> None:
        """hipEventDestroy: frees an event this process created, or closes an
        interprocess event it opened with ``event_open_handle``."""
        _check(self.lib.rnb_event_destroy(ev), "hipEventDestroy")

    def memcpy_async(self, dst: int, src: int, nbytes: int, stream: int) -> None:
        _check(self.lib.rnb_memcpy_async(dst, src, nbytes, stream), "hipMemcpyAsync")

    def memcpy_d2h(self, dst: int, src: int, nbytes: int) -> None:
        _check(self.lib.rnb_memcpy_d2h(dst, src, nbytes), "hipMemcpy D2H")

    def memcpy_peer_async(self, dst, dst_dev, src, src_dev, nbytes, stream) -> None:
        _check(self.lib.rnb_memcpy_peer_async(dst, dst_dev, src, src_dev, nbytes, stream),
               "hipMemcpyPeerAsync")

    def stream_synchronize(self, stream: int) -> None:
        _check(self.lib.rnb_stream_synchronize(stream), "hipStreamSynchronize")

    def can_access_peer(self, dev: int, peer: int) -> bool:
        out = ctypes.c_int()
        _check(self.lib.rnb_can_access_peer(dev, peer, ctypes.byref(out)),
               "hipDeviceCanAccessPeer")
        return bool(out.value)

    def mem_info(self):
        f, t = ctypes.c_size_t(), ctypes.c_size_t()
        _check(self.lib.rnb_mem_get_info(ctypes.byref(f), ctypes.byref(t)), "hipMemGetInfo")
        return f.value, t.value


_kernels: Optional[Kernels] = None
_runtime: Optional[Runtime] = None


def kernels() -> Kernels:
    global _kernels
    if _kernels is None:
        _kernels = Kernels()
    return _kernels


def runtime() -> Runtime:
    global _runtime
    if _runtime is None:
        _runtime = Runtime()
    return _runtime
