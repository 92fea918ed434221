"""C ABI checks without a GPU: the library loads, exports every function declared in
include/*.h, the synthetic weight generator is bit-exact with the oracle, and the
model-dir / argument error paths map onto ClipError variants (src/error.rs:9-41)."""
import ctypes
import glob
import json
import os
import re

import numpy as np
import pytest

from oracle import weights
from oracle.model_spec import TINY_CFG, TINY_SIGLIP_CFG, VIT_B_32_CFG, text_spec_from_cfg, vision_spec_from_cfg
from tests.helpers import make_model_dir

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def declared_functions():
    names = set()
    for h in glob.glob(os.path.join(ROOT, "include", "*.h")):
        src = open(h).read()
        src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
        for m in re.finditer(r"\b(clipgpu_[a-z0-9_]+)\s*\(", src):
            names.add(m.group(1))
    return names


def test_library_exports_every_declared_symbol():
    from open_clip_inference import _lib
    L = _lib.lib()
    names = declared_functions()
    assert len(names) >= 25
    missing = [n for n in names if not hasattr(L, n)]
    assert not missing, missing
    assert set(_lib.SYMBOLS) == names  # the ctypes binding covers exactly the headers
    assert L.clipgpu_abi_version() == 4


def test_no_oracle_in_product():
    """The product package never imports the oracle (test infrastructure only)."""
    pkg = os.path.join(ROOT, "clip-embedder-rs_amd")
    for f in glob.glob(os.path.join(pkg, "**", "*.*"), recursive=True):
        if f.endswith((".py", ".cpp", ".hip", ".hpp", ".h")):
            assert "oracle" not in open(f, errors="ignore").read().replace("oracle/", ""), f


@pytest.mark.parametrize("cfg", [TINY_CFG, VIT_B_32_CFG])
def test_synth_matches_oracle(cfg):
    from open_clip_inference import _lib
    L = _lib.lib()
    v, t = vision_spec_from_cfg(cfg["model_cfg"]), text_spec_from_cfg(cfg["model_cfg"])
    params = weights.vision_param_list(v) + weights.text_param_list(t)
    for name, shape, std, off in params[:40] + params[-10:]:
        ref = weights.synth_tensor(1234, name, shape, std, off).ravel()
        out = np.empty(ref.size, np.float32)
        _lib.check(L.clipgpu_synth_tensor(1234, name.encode(), std, off, out.ctypes.data, out.size))
        assert np.array_equal(ref.view(np.uint32), out.view(np.uint32)), name


def test_create_errors_without_gpu(tmp_path):
    from open_clip_inference.engine import Engine
    from open_clip_inference.error import ConfigError, MissingModelFile, ModelFolderNotFound
    with pytest.raises(ModelFolderNotFound):
        Engine(str(tmp_path / "nope"), 0)
    with pytest.raises(MissingModelFile, match="open_clip_config.json"):
        Engine(str(tmp_path), 0)
    d = make_model_dir(TINY_CFG)
    os.remove(os.path.join(d, "clipgpu_synthetic.json"))
    with pytest.raises(MissingModelFile, match="visual.onnx"):
        Engine(d, 0)
    bad = json.loads(json.dumps(TINY_CFG))
    bad["model_cfg"]["vision_cfg"]["timm_model_name"] = "vit_so400m"
    with pytest.raises(ConfigError, match="not supported"):
        Engine(make_model_dir(bad), 0)
    bad = json.loads(json.dumps(TINY_CFG))
    del bad["preprocess_cfg"]
    with pytest.raises(ConfigError, match="preprocess_cfg"):
        Engine(make_model_dir(bad), 0)


def test_verify_model_dir_mirror(tmp_path):
    from open_clip_inference.error import MissingModelFile, ModelFolderNotFound
    from open_clip_inference.model_manager import MODEL_FILES, get_default_base_folder, verify_model_dir
    assert len(MODEL_FILES) == 9
    assert get_default_base_folder().endswith(os.path.join(".cache", "open_clip_rs"))
    with pytest.raises(ModelFolderNotFound):
        verify_model_dir(str(tmp_path / "x"))
    d = make_model_dir(TINY_CFG)
    verify_model_dir(d)
    with pytest.raises(MissingModelFile, match="tokenizer.json"):
        verify_model_dir(d, need_tokenizer=True)


def test_config_mirror_parses():
    from open_clip_inference.config import ModelConfig, OpenClipConfig
    d = make_model_dir(VIT_B_32_CFG)
    oc = OpenClipConfig.from_file(os.path.join(d, "open_clip_config.json"))
    assert oc.model_cfg.embed_dim == 512 and oc.model_cfg.vision_cfg.image_size == 224
    assert oc.model_cfg.text_cfg.context_length == 77
    assert oc.preprocess_cfg.interpolation == "bicubic" and oc.preprocess_cfg.resize_mode == "shortest"
    mc = ModelConfig.from_file(os.path.join(d, "model_config.json"))
    assert mc.logit_scale == 100.0 and mc.pad_id == 0 and mc.activation_function == "softmax"


def test_safetensors_header_roundtrip(tmp_path):
    """open_clip_model.safetensors is accepted as the weight source (loader runs before
    any device call fails): a wrong-shape file is rejected with a Shape error."""
    from safetensors.numpy import save_file
    from open_clip_inference.engine import Engine
    from open_clip_inference.error import ConfigError
    d = make_model_dir(TINY_CFG)
    os.remove(os.path.join(d, "clipgpu_synthetic.json"))
    save_file({"visual.conv1.weight": np.zeros((3, 3), np.float32)}, os.path.join(d, "open_clip_model.safetensors"))
    with pytest.raises(ConfigError, match="unexpected shape"):
        Engine(d, 0)


@pytest.mark.parametrize("cfg_name", ["TINY_CFG", "TINY_H14_CFG", "TINY_SIGLIP_CFG"])
def test_param_inventory_matches_oracle(cfg_name):
    """csrc/host/weights.cpp tower_params + synth == oracle/weights.py, parameter by parameter
    (names, shapes, init std/offset): bit-exact through the engine's own weight loader."""
    from oracle import model_spec
    from open_clip_inference import _lib
    cfg = getattr(model_spec, cfg_name)
    d = make_model_dir(cfg, seed=4321)
    v, t = vision_spec_from_cfg(cfg["model_cfg"]), text_spec_from_cfg(cfg["model_cfg"])
    for tower, P in ((0, weights.vision_weights(v, 4321)), (1, weights.text_weights(t, 4321))):
        for name, ref in P.items():
            out = np.empty(ref.size, np.float32)
            _lib.check(_lib.lib().clipgpu_test_read_weights(d.encode(), tower, name.encode(), out.ctypes.data,
                                                            out.size))
            assert np.array_equal(out, ref.ravel()), name


@pytest.mark.parametrize("extra,msg", [({"pool_type": "first"}, "pool_type 'first'"),
                                       ({"pool_type": "none"}, "pool_type 'none'"),
                                       ({"proj_type": "mlp"}, "proj_type 'mlp'"),
                                       ({"embed_cls": True}, "embed_cls"),
                                       ({"hf_model_name": "google/siglip"}, "hf_model_name")])
def test_unsupported_text_tower_forms_are_refused(extra, msg):
    """The text engine builds open_clip's TextTransformer in its CLIP form (causal, argmax / EOT
    pooling) and its SigLIP2 form (no_causal_mask, pool_type "last", proj_bias; TINY_SIGLIP_CFG);
    any other text_cfg form (other poolings, MLP projections, CoCa's CLS embedding, HF towers) is
    a Configuration error at clipgpu_create, raised before any device call (runs on CPU)."""
    import json
    from open_clip_inference import _lib
    from open_clip_inference.engine import Engine
    from open_clip_inference.error import ConfigError
    cfg = json.loads(json.dumps(TINY_CFG))
    cfg["model_cfg"]["text_cfg"].update(extra)
    d = make_model_dir(cfg)
    with pytest.raises(ConfigError, match=msg):
        Engine(d, _lib.TOWER_TEXT, [0], "bf16", 8)
    # the CLIP and SigLIP2 forms pass the check (and then fail only for want of a GPU here)
    from oracle.model_spec import TINY_SIGLIP_CFG
    for ok in (TINY_CFG, TINY_SIGLIP_CFG):
        d = make_model_dir(ok)
        try:
            Engine(d, _lib.TOWER_TEXT, [0], "bf16", 8).close()
        except ConfigError as e:  # pragma: no cover
            raise AssertionError(e)
        except Exception:
            pass


def test_library_provenance_is_checked(monkeypatch):
    """The loader refuses a library built from sources other than the tree's (a stale
    lib/libclipgpu.so travels with the tree to the GPU box)."""
    from open_clip_inference import _lib, _source_hash
    from open_clip_inference.error import ClipError
    L = _lib.lib()
    assert L.clipgpu_build_source_hash().decode() == _source_hash.source_hash(os.path.dirname(os.path.dirname(
        os.path.abspath(_lib.__file__))))
    monkeypatch.setattr(_source_hash, "source_hash", lambda d: "0" * 64)
    with pytest.raises(ClipError, match="stale native library"):
        _lib._check_provenance(L)


def _built_tiles():
    """kernels.hpp kGemmTiles: the GemmTile ids the library builds."""
    hdr = open(os.path.join(ROOT, "clip-embedder-rs_amd", "csrc", "kernels", "kernels.hpp")).read()
    ids = {m.group(1): int(m.group(2)) for m in re.finditer(r"\b(TILE_\w+)\s*=\s*(\d+)", hdr)}
    body = re.search(r"kGemmTiles\[\]\s*=\s*\{([^}]*)\}", hdr).group(1)
    return [ids[n.strip()] for n in body.split(",") if n.strip()]


def test_bench_names_every_gemm_tile():
    """bench.py reports the tiles by name: its table covers every GemmTile id the library builds
    (kernels.hpp kGemmTiles), so a new tile cannot crash the bench line; the GPU tests' tile lists
    cover exactly the built tiles."""
    import importlib.util
    built = _built_tiles()
    spec = importlib.util.spec_from_file_location("bench_mod", os.path.join(ROOT, "bench.py"))
    bench = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(bench)
    assert set(built) | {0} <= set(bench.TILE_NAMES)
    for f in ("test_gpu_kernels.py", "test_gpu_parity.py"):
        src = open(os.path.join(ROOT, "tests", f)).read()
        listed = re.search(r"BUILT_TILES = \[([^\]]*)\]", src).group(1)
        assert sorted(int(x) for x in listed.split(",")) == sorted(built), f


def test_engine_reads_no_environment():
    """ABI v3+: every engine behaviour is a clipgpu_options field; the product sources read no
    environment variable (the kernel-level test hooks in testing.hip take CLIPGPU_TEST_TILE only)."""
    csrc = os.path.join(ROOT, "clip-embedder-rs_amd", "csrc")
    for dirpath, _, files in os.walk(csrc):
        for f in files:
            if f.endswith((".hip", ".cpp", ".hpp")) and f != "testing.hip":
                src = open(os.path.join(dirpath, f)).read()
                assert "getenv(" not in src, os.path.join(dirpath, f)


def test_options_init_and_validation():
    """clipgpu_options (per-engine MX split, lanes, tuning, communicator): clipgpu_options_init
    fills the defaults; bad values are refused by clipgpu_create_ex before any device call."""
    from open_clip_inference import _lib
    from open_clip_inference.engine import Engine, Options, mx_site_bits
    from open_clip_inference.error import ClipError, ConfigError
    o = Options()
    _lib.check(_lib.lib().clipgpu_options_init(ctypes.byref(o)))
    assert o.struct_size == ctypes.sizeof(Options) and o.mx_sites == 0 and o.lanes == 0
    assert o.tuning == 0 and o.communicator == 0
    assert mx_site_bits("qkv") == 1 and mx_site_bits(["fc", "proj"]) == 6 and mx_site_bits(None) == 0
    with pytest.raises(ValueError):
        mx_site_bits("attn")
    d = make_model_dir(TINY_CFG)
    for kw, msg in (({"lanes": 5}, "lanes"), ({"mx_sites": "qkv"}, "needs dtype")):
        with pytest.raises(ClipError, match=msg):
            Engine(d, 0, [0], "bf16", 8, **kw)
    with pytest.raises(ClipError, match="proj in MX needs fc"):
        Engine(d, 0, [0], "fp8", 8, mx_sites="qkv,proj")
    for kw, msg in (({"gemm_tiles": [4, 0, 0, 0]}, "not a GEMM tile"), ({"patch_tile": 19}, "not a GEMM tile"),
                    ({"mx_layers": [0, 3]}, "mx_layers needs dtype"), ({"tuning": 3}, "tuning must be")):
        with pytest.raises(ClipError, match=msg):
            Engine(d, 0, [0], "bf16", 8, **kw)
    with pytest.raises(ValueError):
        Engine(d, 0, [0], "bf16", 8, gemm_tiles=[17, 17])
    o2 = Options()
    _lib.check(_lib.lib().clipgpu_options_init(ctypes.byref(o2)))
    assert (o2.graphs, o2.prune_last, o2.trim_text, list(o2.gemm_tiles), o2.patch_tile, o2.mx_layers) == (
        0, 0, 0, [0, 0, 0, 0], 0, 0)
    o2.graphs = 2
    h = ctypes.c_void_p()
    devs = (ctypes.c_int * 1)(0)
    rc = _lib.lib().clipgpu_create_ex(d.encode(), 0, devs, 1, 0, 8, ctypes.byref(o2), ctypes.byref(h))
    assert rc != 0 and b"graphs" in _lib.lib().clipgpu_last_error()
    # a struct_size the library does not know is refused
    o.struct_size = 1
    h = ctypes.c_void_p()
    devs = (ctypes.c_int * 1)(0)
    rc = _lib.lib().clipgpu_create_ex(d.encode(), 0, devs, 1, 0, 8, ctypes.byref(o), ctypes.byref(h))
    assert rc != 0 and b"struct_size" in _lib.lib().clipgpu_last_error()
    # only the published struct sizes (v2: through `communicator`; v3): not one ending inside a field
    for bad in (Options.graphs.offset + 2, ctypes.sizeof(Options) - 2, 8):
        o.struct_size = bad
        rc = _lib.lib().clipgpu_create_ex(d.encode(), 0, devs, 1, 0, 8, ctypes.byref(o), ctypes.byref(h))
        assert rc != 0 and b"struct_size" in _lib.lib().clipgpu_last_error(), bad
    # mx_layers: a 32-bit mask (Python refuses layer 32+, the library bits beyond the tower's layers)
    for bad in ([32], [40], [0, 33], 1 << 32):
        with pytest.raises(ValueError, match="mx_layers"):
            Engine(d, 0, [0], "fp8", 8, mx_layers=bad)
    # residual stream storage (ABI v4): f32 / f16, f16 only for CLIP-family engines (not SigLIP)
    with pytest.raises(ValueError, match="residual"):
        Engine(d, 0, [0], "bf16", 8, residual="bf16")
    with pytest.raises(ClipError, match="residual = f16"):
        Engine(make_model_dir(TINY_SIGLIP_CFG, 3), 0, [0], "bf16", 8, residual="f16")
    o3 = Options()
    _lib.check(_lib.lib().clipgpu_options_init(ctypes.byref(o3)))
    assert o3.residual == 0
    o3.residual = 3
    rc = _lib.lib().clipgpu_create_ex(d.encode(), 0, devs, 1, 0, 8, ctypes.byref(o3), ctypes.byref(h))
    assert rc != 0 and b"residual" in _lib.lib().clipgpu_last_error()
    # LayerNorm fold (ABI v4): -1 / 0 / 1; on only with the f16 stream and a QuickGELU / GELU MLP
    assert o3.ln_fold == 0
    o3.residual = 0
    o3.ln_fold = 2
    rc = _lib.lib().clipgpu_create_ex(d.encode(), 0, devs, 1, 0, 8, ctypes.byref(o3), ctypes.byref(h))
    assert rc != 0 and b"ln_fold" in _lib.lib().clipgpu_last_error()
    with pytest.raises(ClipError, match="ln_fold = 1"):
        Engine(d, 0, [0], "bf16", 8, residual="f32", ln_fold=True)
    with pytest.raises(ClipError, match="ln_fold = 1"):
        Engine(d, 0, [0], "fp8", 8, ln_fold=True)
    tiny_layers = json.load(open(os.path.join(d, "open_clip_config.json")))["model_cfg"]["vision_cfg"]["layers"]
    with pytest.raises(ClipError, match="beyond the tower"):
        Engine(d, 0, [0], "fp8", 8, mx_layers=[tiny_layers])


@pytest.mark.parametrize("rows,off,equal", [([256, 256], [0, 256, 512], 1),
                                            ([3, 0, 5], [0, 3, 3, 8], 0),
                                            ([0, 7], [0, 0, 7], 0),
                                            ([1000, 1000, 1000], [0, 1000, 2000, 3000], 1),
                                            ([5], [0, 5], 1)])
def test_gather_plan(rows, off, equal):
    """The gathered entry points' host-side plan (engine.hip plan_gather): rank-order offsets of
    every rank's block, and the all-gather (equal blocks) vs one-broadcast-per-block choice, incl.
    zero-row ranks and blocks larger than max_batch (chunked per rank; offsets are per rank)."""
    from open_clip_inference import _lib
    n = len(rows)
    r = (ctypes.c_int64 * n)(*rows)
    o = (ctypes.c_int64 * (n + 1))()
    e = ctypes.c_int()
    _lib.check(_lib.lib().clipgpu_test_gather_plan(n, r, o, ctypes.byref(e)))
    assert list(o) == off and e.value == equal


def test_gather_plan_errors():
    from open_clip_inference import _lib
    from open_clip_inference.error import ClipError
    o = (ctypes.c_int64 * 3)()
    e = ctypes.c_int()
    with pytest.raises(ClipError, match="Empty batch"):
        _lib.check(_lib.lib().clipgpu_test_gather_plan(2, (ctypes.c_int64 * 2)(0, 0), o, ctypes.byref(e)))
    with pytest.raises(ClipError, match="negative"):
        _lib.check(_lib.lib().clipgpu_test_gather_plan(2, (ctypes.c_int64 * 2)(4, -1), o, ctypes.byref(e)))


def test_host_register_argument_errors():
    """clipgpu_host_register / _unregister refuse a NULL or empty range and an unknown pointer
    before touching HIP (the registration itself needs a GPU: tests/test_gpu_api.py)."""
    from open_clip_inference import _lib
    from open_clip_inference.error import ClipError
    buf = np.zeros(64, np.uint8)
    with pytest.raises(ClipError, match="NULL / empty"):
        _lib.check(_lib.lib().clipgpu_host_register(None, 64))
    with pytest.raises(ClipError, match="NULL / empty"):
        _lib.check(_lib.lib().clipgpu_host_register(buf.ctypes.data, 0))
    with pytest.raises(ClipError, match="not registered"):
        _lib.check(_lib.lib().clipgpu_host_unregister(buf.ctypes.data))


def test_facade_math_loads_without_hip():
    """Clip.softmax / Clip.sigmoid (host math in the reference, src/clip.rs:172-185) run from the
    host-only library (no HIP, no RCCL in its dependencies), bit-exact to the main library."""
    import subprocess
    from open_clip_inference import _lib
    from open_clip_inference.clip import Clip
    deps = subprocess.run(["ldd", _lib.HOST_LIB_PATH], capture_output=True, text=True).stdout
    assert "amdhip" not in deps and "rccl" not in deps, deps
    x = np.array([1.5, -2.0, 0.25, 3.0], np.float32)
    got = Clip.softmax(x)
    ref = np.empty(4, np.float32)
    one = np.ones(1, np.float32)
    _lib.check(_lib.lib().clipgpu_facade_scores(x.ctypes.data, 4, one.ctypes.data, 1, 1.0, 0.0, 0, ref.ctypes.data))
    assert np.array_equal(got, ref)
    assert Clip.sigmoid(0.0) == 0.5
