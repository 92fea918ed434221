"""Thin owners of the native handles: ``Engine`` (one tower on N GPUs, replaces
``OnnxSession``, src/onnx.rs:7-47) and ``Tokenizer`` (replaces
``tokenizers::Tokenizer`` as configured in src/text.rs:62-85)."""
from __future__ import annotations

import ctypes
from ctypes import POINTER, c_char_p, c_int, c_void_p
from typing import Optional, Sequence

import numpy as np

from . import _lib
from ._lib import check, f3, lib


class Options(ctypes.Structure):
    """``clipgpu_options`` (include/clipgpu.h, ABI v4): per-engine settings of clipgpu_create_ex.  The
    library reads no environment variables: every engine behaviour is one of these fields."""
    _fields_ = [("struct_size", ctypes.c_uint32), ("mx_sites", ctypes.c_uint32), ("lanes", ctypes.c_int32),
                ("tuning", ctypes.c_int32), ("communicator", ctypes.c_int32),
                ("graphs", ctypes.c_int32), ("prune_last", ctypes.c_int32), ("trim_text", ctypes.c_int32),
                ("gemm_tiles", ctypes.c_int32 * 4), ("patch_tile", ctypes.c_int32), ("mx_layers", ctypes.c_uint32),
                ("residual", ctypes.c_int32), ("ln_fold", ctypes.c_int32)]


def _tristate(v) -> int:
    """None -> 0 (the default), True -> 1, False -> -1 (clipgpu_options on/off fields)."""
    return 0 if v is None else (1 if v else -1)


MX_SITE_BITS = {"qkv": 1, "fc": 2, "proj": 4}  # CLIPGPU_MX_QKV / _FC / _PROJ


def mx_site_bits(sites) -> int:
    """"qkv,fc" / ["qkv", "fc"] -> CLIPGPU_MX_* bits (0 = the default split)."""
    if sites is None:
        return 0
    if isinstance(sites, str):
        sites = [s for s in sites.split(",") if s]
    bits = 0
    for s in sites:
        if s not in MX_SITE_BITS:
            raise ValueError(f"unknown MX site {s!r}: one of {sorted(MX_SITE_BITS)}")
        bits |= MX_SITE_BITS[s]
    return bits


class Engine:
    def __init__(self, model_dir: str, tower: int, devices: Optional[Sequence[int]] = None,
                 dtype: str = "bf16", max_batch: int = 256, mx_sites=None, lanes: int = 0, tuning=False,
                 communicator: bool = False, graphs: Optional[bool] = None, prune_last: Optional[bool] = None,
                 trim_text: Optional[bool] = None, gemm_tiles: Optional[Sequence[int]] = None, patch_tile: int = 0,
                 mx_layers=None, residual: Optional[str] = None, ln_fold: Optional[bool] = None):
        """mx_sites: fp8 engines' MX split ("qkv,fc,proj" by default); lanes: concurrent sub-batch lanes
        (0 = the tile table's); tuning: time the GEMM tiles at creation instead of the committed table
        (True / 1: per site + whole forwards, 2: per site only); communicator: create a multi-device
        handle's RCCL communicator now, not on the first gather; graphs / prune_last / trim_text: None =
        the default (on), False = off (all bit-identical); gemm_tiles: [qkv, out_proj, c_fc, c_proj]
        GemmTile ids (0 = the table's, -1 = the shape heuristic), patch_tile likewise; mx_layers: fp8
        engines' layers that run their MX sites in MX-fp8 (a bit mask or a list of layer indices;
        None = every layer); residual: the residual stream's storage, "f32" or "f16" (None = the
        library's default); ln_fold: ln_1 / ln_2 folded into the QKV / c_fc GEMMs (None = where it
        applies, True = required, False = LayerNorm kernels)."""
        self.model_dir = model_dir
        self.tower = tower
        self.devices = list(devices) if devices else [0]
        self.dtype = dtype
        self.max_batch = int(max_batch)
        self.opts = {"mx_sites": mx_sites, "lanes": int(lanes), "tuning": tuning, "communicator": bool(communicator),
                     "graphs": graphs, "prune_last": prune_last, "trim_text": trim_text,
                     "gemm_tiles": list(gemm_tiles) if gemm_tiles else None, "patch_tile": int(patch_tile),
                     "mx_layers": mx_layers, "residual": residual,
                     "ln_fold": ln_fold}  # duplicate() rebuilds with the same
        dt = {"bf16": _lib.DTYPE_BF16, "f16": _lib.DTYPE_F16, "fp16": _lib.DTYPE_F16, "fp8": _lib.DTYPE_FP8}[dtype]
        devs = (c_int * len(self.devices))(*self.devices)
        opts = Options()
        check(lib().clipgpu_options_init(ctypes.byref(opts)))
        opts.mx_sites = mx_site_bits(mx_sites)
        opts.lanes = int(lanes)
        opts.tuning = int(tuning) if not isinstance(tuning, bool) else (1 if tuning else 0)
        opts.communicator = 1 if communicator else 0
        opts.graphs = _tristate(graphs)
        opts.prune_last = _tristate(prune_last)
        opts.trim_text = _tristate(trim_text)
        if gemm_tiles:
            if len(gemm_tiles) != 4:
                raise ValueError("gemm_tiles: four GemmTile ids (qkv, out_proj, c_fc, c_proj)")
            for i, t in enumerate(gemm_tiles):
                opts.gemm_tiles[i] = int(t)
        opts.patch_tile = int(patch_tile)
        if mx_layers is not None:
            if not isinstance(mx_layers, int):
                layers = [int(l) for l in mx_layers]
                if any(l < 0 or l >= 32 for l in layers):
                    raise ValueError("mx_layers: layer indices 0..31 (clipgpu_options.mx_layers is a 32-bit mask)")
                mx_layers = sum(1 << l for l in set(layers))
            if mx_layers < 0 or mx_layers > 0xFFFFFFFF:
                raise ValueError("mx_layers: a 32-bit layer mask (clipgpu_options.mx_layers)")
            if mx_layers == 0:
                raise ValueError("mx_layers: at least one layer (None = every layer)")
            opts.mx_layers = int(mx_layers)
        if residual not in (None, "f32", "f16"):
            raise ValueError('residual: "f32" or "f16"')
        opts.residual = {None: 0, "f32": 1, "f16": 2}[residual]
        opts.ln_fold = _tristate(ln_fold)
        h = c_void_p()
        check(lib().clipgpu_create_ex(model_dir.encode(), tower, devs, len(self.devices), dt, self.max_batch,
                                      ctypes.byref(opts), ctypes.byref(h)))
        self._h = h

    def info(self):
        """(tiles per trunk site [qkv, out_proj, c_fc, c_proj], device lanes, MX site names)."""
        tiles = (c_int * 4)()
        lanes = c_int()
        bits = ctypes.c_uint32()
        check(lib().clipgpu_engine_info(self.handle, tiles, ctypes.byref(lanes), ctypes.byref(bits)))
        sites = [s for s, b in MX_SITE_BITS.items() if bits.value & b]
        return list(tiles), lanes.value, sites

    @property
    def handle(self):
        if self._h is None:
            raise RuntimeError("engine destroyed")
        return self._h

    def close(self):
        if getattr(self, "_h", None) is not None:
            lib().clipgpu_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    @property
    def embed_dim(self) -> int:
        return lib().clipgpu_embed_dim(self.handle)

    @property
    def input_size(self) -> int:
        return lib().clipgpu_input_size(self.handle)

    def _out(self, B: int, out: Optional[np.ndarray]) -> np.ndarray:
        # `out`: an optional caller [B, embed_dim] float32 C-contiguous array (e.g. a registered one)
        if out is None:
            return np.empty((B, self.embed_dim), np.float32)
        if out.dtype != np.float32 or out.shape != (B, self.embed_dim) or not out.flags["C_CONTIGUOUS"]:
            raise ValueError(f"out must be a C-contiguous float32 [{B}, {self.embed_dim}] array")
        return out

    def embed_pixels(self, nchw: np.ndarray, out: Optional[np.ndarray] = None) -> np.ndarray:
        x = np.ascontiguousarray(nchw, dtype=np.float32)
        if x.ndim != 4 or x.shape[1] != 3 or x.shape[2] != x.shape[3]:
            from .error import ShapeError
            raise ShapeError(f"Shape error: expected [B,3,S,S], got {x.shape}")
        out = self._out(x.shape[0], out)
        check(lib().clipgpu_embed_pixels(self.handle, x.ctypes.data, x.shape[0], x.shape[2], out.ctypes.data))
        return out

    def embed_u8(self, nhwc: np.ndarray, mean, std, out: Optional[np.ndarray] = None) -> np.ndarray:
        x = np.ascontiguousarray(nhwc, dtype=np.uint8)
        out = self._out(x.shape[0], out)
        check(lib().clipgpu_embed_u8(self.handle, x.ctypes.data, x.shape[0], x.shape[1], f3(mean), f3(std),
                                     out.ctypes.data))
        return out

    def embed_images_rgb8(self, images) -> np.ndarray:
        """Decoded RGB8 images (HxWx3 uint8, any sizes) -> embeddings, crop/resize/normalise on
        the GPU with the model folder's preprocess_cfg (clipgpu_embed_images_rgb8)."""
        arrs = [np.ascontiguousarray(a, dtype=np.uint8) for a in images]
        n = len(arrs)
        for a in arrs:
            if a.ndim != 3 or a.shape[2] != 3:
                from .error import ShapeError
                raise ShapeError(f"Shape error: expected [H,W,3] uint8, got {a.shape}")
        ptrs = (c_void_p * max(n, 1))(*[a.ctypes.data for a in arrs])
        ws = (c_int * max(n, 1))(*[a.shape[1] for a in arrs])
        hs = (c_int * max(n, 1))(*[a.shape[0] for a in arrs])
        out = np.empty((n, self.embed_dim), np.float32)
        check(lib().clipgpu_embed_images_rgb8(self.handle, ptrs, ws, hs, n, out.ctypes.data))
        return out

    def embed_tokens(self, ids: np.ndarray, mask: Optional[np.ndarray] = None,
                     out: Optional[np.ndarray] = None) -> np.ndarray:
        x = np.ascontiguousarray(ids, dtype=np.int64)
        m = None if mask is None else np.ascontiguousarray(mask, dtype=np.int64)
        out = self._out(x.shape[0], out)
        check(lib().clipgpu_embed_tokens(self.handle, x.ctypes.data, None if m is None else m.ctypes.data,
                                         x.shape[0], x.shape[1], out.ctypes.data))
        return out

    # Device-resident variants: raw device pointers (ints), stream = hipStream_t or 0 (the legacy
    # default stream, torch's default: the forward is ordered on it, include/clipgpu.h).
    def embed_pixels_device(self, d_in: int, B: int, d_out: int, stream: int = 0) -> None:
        check(lib().clipgpu_embed_pixels_device(self.handle, c_void_p(d_in), B, c_void_p(d_out),
                                                c_void_p(stream or None)))

    def embed_u8_device(self, d_in: int, B: int, mean, std, d_out: int, stream: int = 0) -> None:
        check(lib().clipgpu_embed_u8_device(self.handle, c_void_p(d_in), B, f3(mean), f3(std), c_void_p(d_out),
                                            c_void_p(stream or None)))

    def embed_tokens_device(self, d_ids: int, B: int, d_out: int, stream: int = 0) -> None:
        check(lib().clipgpu_embed_tokens_device(self.handle, c_void_p(d_ids), B, c_void_p(d_out),
                                                c_void_p(stream or None)))

    # ---- data-parallel sharding + the RCCL all-gather (include/clipgpu.h) ----------------
    @staticmethod
    def comm_unique_id() -> bytes:
        buf = (ctypes.c_uint8 * 128)()
        check(lib().clipgpu_comm_unique_id(buf))
        return bytes(buf)

    def comm_init_rank(self, uid: bytes, nranks: int, rank: int) -> None:
        if len(uid) != 128:
            raise ValueError("the unique id is 128 bytes")
        buf = (ctypes.c_uint8 * 128).from_buffer_copy(uid)
        check(lib().clipgpu_comm_init_rank(self.handle, buf, int(nranks), int(rank)))

    def comm_info(self):
        n, r0 = c_int(), c_int()
        check(lib().clipgpu_comm_info(self.handle, ctypes.byref(n), ctypes.byref(r0)))
        return n.value, r0.value

    def _gather(self, fn, d_in, rows, d_out, streams):
        k = len(self.devices)
        if len(d_in) != k or len(d_out) != k:
            raise ValueError(f"one input and one output buffer per local device ({k})")
        ins = (c_void_p * k)(*[c_void_p(p) for p in d_in])
        outs = (c_void_p * k)(*[c_void_p(p) for p in d_out])
        rs = (ctypes.c_int64 * len(rows))(*[int(r) for r in rows])
        # streams None: a NULL array (every device's legacy default stream, as a NULL entry is)
        sts = None if streams is None else (c_void_p * k)(*[c_void_p(s or None) for s in streams])
        check(fn(self.handle, ins, rs, outs, sts))

    def embed_pixels_gather_device(self, d_in, rows, d_out, streams=None) -> None:
        """Per local device: its rank's block of normalised pixels in, the whole [sum rows][E]
        embedding matrix (rank order) out -- forward + one RCCL all-gather."""
        self._gather(lib().clipgpu_embed_pixels_gather_device, d_in, rows, d_out, streams)

    def embed_tokens_gather_device(self, d_in, rows, d_out, streams=None) -> None:
        self._gather(lib().clipgpu_embed_tokens_gather_device, d_in, rows, d_out, streams)


PROFILE_CATEGORIES = ["patch_embed", "stem_ln", "qkv", "attention", "out_proj", "layernorm", "c_fc",
                      "c_proj", "head", "last_layer"]


PROFILE_CONCURRENT = 0x80000000  # include/clipgpu.h CLIPGPU_PROFILE_CONCURRENT: keep the lanes concurrent


def profile_enable(engine: "Engine", categories, concurrent: bool = False) -> None:
    mask = PROFILE_CONCURRENT if concurrent and categories else 0
    for c in categories:
        mask |= 1 << PROFILE_CATEGORIES.index(c)
    check(lib().clipgpu_profile_enable(engine.handle, mask))


def profile_read(engine: "Engine", category: str):
    ms = ctypes.c_double()
    n = ctypes.c_int64()
    check(lib().clipgpu_profile_read(engine.handle, PROFILE_CATEGORIES.index(category), ctypes.byref(ms),
                                     ctypes.byref(n)))
    return ms.value, n.value


def host_buffer(shape, dtype) -> np.ndarray:
    """An empty C-contiguous host array that owns whole memory pages (page-aligned start, no other
    allocation on its last page): what host_register needs, since registration pins whole pages and two
    registered ranges may not share one (clipgpu_host_register)."""
    dtype = np.dtype(dtype)
    n = int(np.prod(shape, dtype=np.int64)) * dtype.itemsize
    page = 4096
    raw = np.empty(((n + page - 1) // page + 1) * page, np.uint8)
    off = (-raw.ctypes.data) % page
    return raw[off:off + n].view(dtype).reshape(shape)


def host_register(arr: np.ndarray) -> None:
    """Registers a C-contiguous host array for direct DMA by the host-buffer entry points
    (clipgpu_host_register).  Keep `arr` alive until host_unregister(arr).  A range that shares a memory
    page with a registered one is refused: allocate registered arrays with host_buffer."""
    if not arr.flags["C_CONTIGUOUS"]:
        raise ValueError("host_register needs a C-contiguous array")
    check(lib().clipgpu_host_register(arr.ctypes.data, arr.nbytes))


def host_unregister(arr: np.ndarray) -> None:
    check(lib().clipgpu_host_unregister(arr.ctypes.data))


class Tokenizer:
    def __init__(self, tokenizer_json: str, context_length: int, pad_id: Optional[int] = None):
        h = c_void_p()
        check(lib().clipgpu_tokenizer_create(tokenizer_json.encode(), int(context_length),
                                             -1 if pad_id is None else int(pad_id), ctypes.byref(h)))
        self._h = h
        self.context_length = int(context_length)

    def close(self):
        if getattr(self, "_h", None) is not None:
            lib().clipgpu_tokenizer_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def token_id(self, tok: str) -> Optional[int]:
        v = lib().clipgpu_tokenizer_token_id(self._h, tok.encode("utf-8"))
        return None if v < 0 else int(v)

    @property
    def vocab_size(self) -> int:
        return int(lib().clipgpu_tokenizer_vocab_size(self._h))

    def encode_batch(self, texts: Sequence[str], lowercase: bool = False):
        n = len(texts)
        enc = [t.encode("utf-8") for t in texts]
        arr = (c_char_p * max(n, 1))(*enc)
        lens = np.array([len(e) for e in enc] or [0], np.int64)
        ids = np.empty((n, self.context_length), np.int64)
        mask = np.empty((n, self.context_length), np.int64)
        check(lib().clipgpu_tokenize(self._h, arr, lens.ctypes.data, n, 1 if lowercase else 0, ids.ctypes.data,
                                     mask.ctypes.data))
        return ids, mask


RESIZE_IMPLS = ("fast_image_resize", "image")  # src/vision.rs:149-157: the crate feature picks one


def resize_rgb8(rgb: np.ndarray, size: int, interpolation: str = "bicubic", resize_mode: str = "shortest",
                resize_impl: str = "fast_image_resize"):
    """resize_with_fast_image_resize (default, src/vision.rs:164-198) or resize_with_image
    (resize_impl="image", src/vision.rs:200-233)."""
    x = np.ascontiguousarray(rgb, dtype=np.uint8)
    out = np.empty((size, size, 3), np.uint8)
    fn = lib().clipgpu_resize_rgb8_image if resize_impl == "image" else lib().clipgpu_resize_rgb8
    check(fn(x.ctypes.data, x.shape[1], x.shape[0], size, interpolation.encode(), resize_mode.encode(),
             out.ctypes.data))
    return out


SIM_ACTIVATIONS = {"softmax": 0, "sigmoid": 1, "logits": 2}


def similarity(img_embs: np.ndarray, txt_embs: np.ndarray, logit_scale: float = 1.0, logit_bias: float = 0.0,
               activation: str = "softmax", axis: int = 1, device: int = 0) -> np.ndarray:
    """src/clip.rs:79-185 arithmetic for [n_img, E] x [n_txt, E] on the GPU
    (clipgpu_similarity): [n_img, n_txt] logits / sigmoid / softmax along `axis`."""
    a = np.ascontiguousarray(img_embs, dtype=np.float32)
    b = np.ascontiguousarray(txt_embs, dtype=np.float32)
    if a.ndim != 2 or b.ndim != 2 or a.shape[1] != b.shape[1]:
        from .error import ShapeError
        raise ShapeError(f"Shape error: {a.shape} vs {b.shape}")
    out = np.empty((a.shape[0], b.shape[0]), np.float32)
    check(lib().clipgpu_similarity(int(device), a.ctypes.data, a.shape[0], b.ctypes.data, b.shape[0], a.shape[1],
                                   float(logit_scale), float(logit_bias), SIM_ACTIVATIONS[activation], int(axis),
                                   out.ctypes.data))
    return out


def resize_rgb8_gpu(images, size: int, interpolation: str = "bicubic", resize_mode: str = "shortest"):
    """The GPU crop/resize alone (test hook): [n, size, size, 3] uint8."""
    arrs = [np.ascontiguousarray(a, dtype=np.uint8) for a in images]
    n = len(arrs)
    ptrs = (c_void_p * max(n, 1))(*[a.ctypes.data for a in arrs])
    ws = (c_int * max(n, 1))(*[a.shape[1] for a in arrs])
    hs = (c_int * max(n, 1))(*[a.shape[0] for a in arrs])
    out = np.empty((n, size, size, 3), np.uint8)
    check(lib().clipgpu_test_resize_rgb8_gpu(ptrs, ws, hs, n, size, interpolation.encode(), resize_mode.encode(),
                                             out.ctypes.data))
    return out


def preprocess_batch_rgb8(images, size: int, interpolation: str, resize_mode: str, mean, std,
                          resize_impl: str = "fast_image_resize") -> np.ndarray:
    if resize_impl not in RESIZE_IMPLS:
        raise ValueError(f"resize_impl must be one of {RESIZE_IMPLS}")
    arrs = [np.ascontiguousarray(a, dtype=np.uint8) for a in images]
    n = len(arrs)
    out = np.empty((n, 3, size, size), np.float32)
    ptrs = (c_void_p * max(n, 1))(*[a.ctypes.data for a in arrs])
    ws = (c_int * max(n, 1))(*[a.shape[1] for a in arrs])
    hs = (c_int * max(n, 1))(*[a.shape[0] for a in arrs])
    fn = lib().clipgpu_preprocess_batch_image if resize_impl == "image" else lib().clipgpu_preprocess_batch
    check(fn(ptrs, ws, hs, n, size, interpolation.encode(), resize_mode.encode(), f3(mean), f3(std), out.ctypes.data))
    return out
