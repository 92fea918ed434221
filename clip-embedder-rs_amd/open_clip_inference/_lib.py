"""ctypes binding of ``include/clipgpu.h`` (the C ABI of ``lib/libclipgpu.so``).

The shared library is the product: HIP/gfx950 kernels + C++ host runtime.  There
is no fallback — if the library is missing or fails to load, every entry point
raises, loudly.
"""
from __future__ import annotations

import ctypes
import os
from ctypes import POINTER, c_char_p, c_double, c_float, c_int, c_int64, c_uint64, c_void_p

from .error import ClipError, error_for_status

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("CLIPGPU_LIB", os.path.join(os.path.dirname(_HERE), "lib", "libclipgpu.so"))

TOWER_VISION = 0
TOWER_TEXT = 1
DTYPE_BF16 = 0
DTYPE_F16 = 1
DTYPE_FP8 = 2  # MX-fp8 trunk GEMMs (BASELINE configs[4] "fp8 MFMA weight path")

# (name, restype, argtypes) — every symbol declared in include/clipgpu.h.
_PROTOS = [
    ("clipgpu_last_error", c_char_p, []),
    ("clipgpu_abi_version", c_int, []),
    ("clipgpu_build_source_hash", c_char_p, []),
    ("clipgpu_create", c_int, [c_char_p, c_int, POINTER(c_int), c_int, c_int, c_int, POINTER(c_void_p)]),
    ("clipgpu_options_init", c_int, [c_void_p]),
    ("clipgpu_create_ex", c_int, [c_char_p, c_int, POINTER(c_int), c_int, c_int, c_int, c_void_p, POINTER(c_void_p)]),
    ("clipgpu_engine_info", c_int, [c_void_p, POINTER(c_int), POINTER(c_int), POINTER(ctypes.c_uint32)]),
    ("clipgpu_destroy", None, [c_void_p]),
    ("clipgpu_embed_dim", c_int, [c_void_p]),
    ("clipgpu_input_size", c_int, [c_void_p]),
    ("clipgpu_num_devices", c_int, [c_void_p]),
    ("clipgpu_embed_pixels", c_int, [c_void_p, c_void_p, c_int64, c_int64, c_void_p]),
    ("clipgpu_embed_u8", c_int, [c_void_p, c_void_p, c_int64, c_int64, POINTER(c_float), POINTER(c_float), c_void_p]),
    ("clipgpu_host_register", c_int, [c_void_p, ctypes.c_size_t]),
    ("clipgpu_host_unregister", c_int, [c_void_p]),
    ("clipgpu_embed_tokens", c_int, [c_void_p, c_void_p, c_void_p, c_int64, c_int64, c_void_p]),
    ("clipgpu_embed_pixels_device", c_int, [c_void_p, c_void_p, c_int64, c_void_p, c_void_p]),
    ("clipgpu_embed_u8_device", c_int, [c_void_p, c_void_p, c_int64, POINTER(c_float), POINTER(c_float), c_void_p, c_void_p]),
    ("clipgpu_embed_tokens_device", c_int, [c_void_p, c_void_p, c_int64, c_void_p, c_void_p]),
    ("clipgpu_embed_images_rgb8", c_int, [c_void_p, POINTER(c_void_p), POINTER(c_int), POINTER(c_int), c_int64, c_void_p]),
    ("clipgpu_preprocess_rgb8", c_int, [c_void_p, c_int, c_int, c_int, c_char_p, c_char_p, POINTER(c_float), POINTER(c_float), c_void_p]),
    ("clipgpu_resize_rgb8", c_int, [c_void_p, c_int, c_int, c_int, c_char_p, c_char_p, c_void_p]),
    ("clipgpu_preprocess_batch", c_int, [POINTER(c_void_p), POINTER(c_int), POINTER(c_int), c_int64, c_int, c_char_p, c_char_p, POINTER(c_float), POINTER(c_float), c_void_p]),
    ("clipgpu_resize_rgb8_image", c_int, [c_void_p, c_int, c_int, c_int, c_char_p, c_char_p, c_void_p]),
    ("clipgpu_preprocess_batch_image", c_int, [POINTER(c_void_p), POINTER(c_int), POINTER(c_int), c_int64, c_int, c_char_p, c_char_p, POINTER(c_float), POINTER(c_float), c_void_p]),
    ("clipgpu_tokenizer_create", c_int, [c_char_p, c_int, c_int64, POINTER(c_void_p)]),
    ("clipgpu_tokenizer_destroy", None, [c_void_p]),
    ("clipgpu_tokenize", c_int, [c_void_p, POINTER(c_char_p), c_void_p, c_int64, c_int, c_void_p, c_void_p]),
    ("clipgpu_tokenizer_token_id", c_int64, [c_void_p, c_char_p]),
    ("clipgpu_tokenizer_vocab_size", c_int64, [c_void_p]),
    ("clipgpu_similarity", c_int, [c_int, c_void_p, c_int64, c_void_p, c_int64, c_int64, c_float, c_float, c_int, c_int, c_void_p]),
    ("clipgpu_similarity_device", c_int, [c_void_p, c_int64, c_void_p, c_int64, c_int64, c_float, c_float, c_int, c_int, c_void_p, c_void_p]),
    ("clipgpu_comm_unique_id", c_int, [c_void_p]),
    ("clipgpu_comm_init_rank", c_int, [c_void_p, c_void_p, c_int, c_int]),
    ("clipgpu_comm_info", c_int, [c_void_p, POINTER(c_int), POINTER(c_int)]),
    ("clipgpu_embed_pixels_gather_device", c_int, [c_void_p, POINTER(c_void_p), POINTER(c_int64), POINTER(c_void_p), POINTER(c_void_p)]),
    ("clipgpu_embed_tokens_gather_device", c_int, [c_void_p, POINTER(c_void_p), POINTER(c_int64), POINTER(c_void_p), POINTER(c_void_p)]),
    ("clipgpu_facade_scores", c_int, [c_void_p, c_int64, c_void_p, c_int64, c_float, c_float, c_int, c_void_p]),
    ("clipgpu_profile_enable", c_int, [c_void_p, ctypes.c_uint]),
    ("clipgpu_profile_read", c_int, [c_void_p, c_int, POINTER(c_double), POINTER(c_int64)]),
    ("clipgpu_profile_category_name", c_char_p, [c_int]),
    ("clipgpu_synth_tensor", c_int, [c_uint64, c_char_p, c_double, c_double, c_void_p, c_int64]),
    # include/clipgpu_testing.h
    ("clipgpu_test_gemm", c_int, [c_int, c_int, c_int, c_int64, c_int64, c_int64, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p]),
    ("clipgpu_test_gemm_chunk_rows", c_int, [c_int64]),
    ("clipgpu_test_gemm_lnf", c_int, [c_int, c_int, c_int64, c_int64, c_int64, c_void_p, c_void_p, c_void_p,
                               c_void_p, c_float, c_int, c_void_p]),
    ("clipgpu_test_attention", c_int, [c_int, c_int64, c_int64, c_int64, c_int64, c_int, c_void_p, c_void_p]),
    ("clipgpu_test_layernorm", c_int, [c_int, c_int64, c_int64, c_float, c_void_p, c_void_p, c_void_p, c_void_p]),
    ("clipgpu_test_gemm_grid", c_int, [c_int, c_int64, c_int64, c_int64, POINTER(c_int)]),
    ("clipgpu_test_gemm_bench", c_int, [c_int, c_int, c_int, c_int64, c_int64, c_int64, c_int, c_int, POINTER(c_double)]),
    ("clipgpu_test_h2d_bench", c_int, [c_int64, c_int, c_int, POINTER(c_double)]),
    ("clipgpu_test_host_copy", c_int, [c_int64, c_int, c_int, POINTER(c_double)]),
    ("clipgpu_test_install_crash_handler", c_int, []),
    ("clipgpu_test_gemm_bench_ld", c_int, [c_int, c_int, c_int, c_int64, c_int64, c_int64, c_int64, c_int64, c_int, c_int,
                                           POINTER(c_double)]),
    ("clipgpu_test_engine_tiles", c_int, [c_void_p, POINTER(c_int)]),
    ("clipgpu_test_engine_lanes", c_int, [c_void_p, POINTER(c_int)]),
    ("clipgpu_test_engine_residual", c_int, [c_void_p, POINTER(c_int), POINTER(c_int)]),
    ("clipgpu_test_host_plan", c_int, [c_void_p, c_int, POINTER(c_int), c_int]),
    ("clipgpu_test_force_broadcast", c_int, [c_void_p, c_int]),
    ("clipgpu_test_rgb8_resize_always", c_int, [c_void_p, c_int]),
    ("clipgpu_test_comm_lazy", c_int, [c_void_p]),
    ("clipgpu_test_profile_timeline", c_int, [c_void_p, c_int64, POINTER(c_double), POINTER(c_double), POINTER(c_int),
                                              POINTER(c_int), POINTER(c_int64)]),
    ("clipgpu_test_gather_plan", c_int, [c_int, POINTER(c_int64), POINTER(c_int64), POINTER(c_int)]),
    ("clipgpu_test_read_weights", c_int, [c_char_p, c_int, c_char_p, c_void_p, c_int64]),
    ("clipgpu_test_patch_embed", c_int, [c_int, c_int, c_int64, c_int64, c_int64, c_int64, c_void_p, POINTER(c_float), POINTER(c_float), c_void_p, c_void_p, c_void_p]),
    ("clipgpu_test_resize_rgb8_gpu", c_int, [POINTER(c_void_p), POINTER(c_int), POINTER(c_int), c_int64, c_int, c_char_p, c_char_p, c_void_p]),
    ("clipgpu_test_lane_reduce", c_int, [c_void_p, c_void_p]),
    ("clipgpu_test_patch_rows", c_int, [c_int, c_int, c_int64, c_int64, c_int64, c_void_p, POINTER(c_float), POINTER(c_float), c_void_p]),
    ("clipgpu_test_clock_probe", c_int, [c_void_p, c_int64, c_void_p]),
    ("clipgpu_test_attention_bench", c_int, [c_int, c_int64, c_int64, c_int64, c_int64, c_int, c_int, POINTER(c_double)]),
    ("clipgpu_test_quant_rows", c_int, [c_int64, c_int64, c_void_p, c_void_p, c_void_p]),
    ("clipgpu_test_layernorm_mx", c_int, [c_int64, c_int64, c_float, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p]),
    ("clipgpu_test_gemm_mx", c_int, [c_int, c_int, c_int, c_int64, c_int64, c_int64, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p]),
    ("clipgpu_test_gemm_mx_bench", c_int, [c_int, c_int, c_int64, c_int64, c_int64, c_int, c_int, POINTER(c_double)]),
]

SYMBOLS = [p[0] for p in _PROTOS]

_lib = None


def lib():
    """Load libclipgpu.so once.  Raises ClipError if it is absent (no fallback)."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise ClipError(f"clipgpu native library not found at {LIB_PATH}; "
                            "run `make -C clip-embedder-rs_amd` (or __graft_entry__.build())")
        L = ctypes.CDLL(LIB_PATH)
        for name, res, args in _PROTOS:
            fn = getattr(L, name)
            fn.restype = res
            fn.argtypes = args
        _check_provenance(L)
        _lib = L
    return _lib


HOST_LIB_PATH = os.path.join(os.path.dirname(LIB_PATH), "libclipgpu_host.so")
_host = None


def host_lib():
    """The host-only library (lib/libclipgpu_host.so: no HIP, no RCCL) with the Clip facade's
    bit-exact score arithmetic (clipgpu_facade_scores, csrc/host/facade.cpp) -- loadable on a
    host without ROCm.  Same provenance check as lib()."""
    global _host
    if _host is None:
        if not os.path.exists(HOST_LIB_PATH):
            raise ClipError(f"clipgpu host library not found at {HOST_LIB_PATH}; run `make -C clip-embedder-rs_amd`")
        L = ctypes.CDLL(HOST_LIB_PATH)
        for name, res, args in _PROTOS:
            if name in ("clipgpu_last_error", "clipgpu_facade_scores", "clipgpu_build_source_hash"):
                fn = getattr(L, name)
                fn.restype = res
                fn.argtypes = args
        _check_provenance(L, HOST_LIB_PATH)
        _host = L
    return _host


def check_host(rc: int) -> None:
    if rc != 0:
        msg = host_lib().clipgpu_last_error().decode("utf-8", "replace")
        raise error_for_status(rc, msg)


def _check_provenance(L, path=LIB_PATH) -> None:
    """The library must have been built from the sources next to it (binary provenance)."""
    from ._source_hash import source_hash
    fn = L.clipgpu_build_source_hash
    fn.restype = c_char_p
    fn.argtypes = []
    built = fn().decode()
    here = source_hash(os.path.dirname(_HERE))
    if built != here:
        raise ClipError(f"stale native library {path}: built from sources {built[:12]}, the tree has "
                        f"{here[:12]}; rebuild with `make -C clip-embedder-rs_amd` (__graft_entry__.build())")


def check(rc: int) -> None:
    if rc != 0:
        msg = lib().clipgpu_last_error().decode("utf-8", "replace")
        raise error_for_status(rc, msg)


def f3(vals):
    return (c_float * 3)(*[float(v) for v in vals])
