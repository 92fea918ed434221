"""The exact configurations `bench.py` measures, checked against the fp64 oracle.

`bench.py`'s headline (BASELINE.json configs[1]) and its text leg (configs[2]) run engines
built exactly as the bench builds them: the bench's own model folder and seeded inputs,
max_batch 256 / 1024, the committed tile table (engine.hip table_tiles / table_lanes: vision two
lanes of 128 images with tiles 15,26,15,15 -- 224x192 8-wave out_proj, 160x128 4-wave RS qkv / c_fc /
c_proj / patch GEMM; text two lanes of 512 sequences with 18,17,18,15),
the hipGraph-replayed device entry point on the caller's stream.  Sampled rows spread over the
batch: the first and last rows, the rows around the 128 / 512 midpoints (where the two lanes of
each tower cut) and rows whose tokens
straddle GEMM row-tile boundaries; every row of the batch is checked for unit norm, and a second
replay must give the same bits.  Tolerance: cosine >= 0.9999 per row (north_star,
tests/helpers.py).
"""
import numpy as np
import pytest

from oracle import clip_ref, weights
from oracle.model_spec import VIT_B_32_CFG, text_spec_from_cfg, vision_spec_from_cfg
from tests.helpers import COS_TOL

pytestmark = pytest.mark.gpu

VISION_ROWS = [0, 1, 63, 126, 127, 128, 129, 191, 254, 255]
TEXT_ROWS = [0, 1, 255, 510, 511, 512, 513, 767, 1022, 1023]


@pytest.fixture(scope="module")
def bench_mod():
    import bench
    assert bench.CFG["model_cfg"] == VIT_B_32_CFG["model_cfg"]
    return bench


def _tiles(engine):
    from ctypes import c_int
    from open_clip_inference import _lib
    t = (c_int * 4)()
    _lib.check(_lib.lib().clipgpu_test_engine_tiles(engine._h, t))
    return list(t)


def test_bench_vision_config_matches_oracle(bench_mod):
    import torch
    from open_clip_inference import _lib
    from open_clip_inference.engine import Engine
    B = bench_mod.B_VISION
    dev = torch.device("cuda", 0)
    ve = Engine(bench_mod.make_model_dir(), _lib.TOWER_VISION, [0], "bf16", B)
    px, _ = bench_mod.synth_inputs(0, dev)
    out = torch.empty((B, 512), device=dev, dtype=torch.float32)
    s = torch.cuda.current_stream(dev)
    ve.embed_pixels_device(px.data_ptr(), B, out.data_ptr(), s.cuda_stream)
    torch.cuda.synchronize()
    first = out.cpu().numpy()
    out.zero_()
    ve.embed_pixels_device(px.data_ptr(), B, out.data_ptr(), s.cuda_stream)  # graph replay
    torch.cuda.synchronize()
    got = out.cpu().numpy()
    assert np.array_equal(first, got)
    assert np.all(np.abs(np.linalg.norm(got, axis=1) - 1) < 1e-5)
    v = vision_spec_from_cfg(VIT_B_32_CFG["model_cfg"])
    ref = clip_ref.encode_image(weights.vision_weights(v, 1234), v, px[VISION_ROWS].cpu().numpy())
    cos = clip_ref.cosine_rows(got[VISION_ROWS], ref)
    print("bench vision tiles", _tiles(ve), "cos min", float(cos.min()))
    assert cos.min() >= COS_TOL, (cos.min(), _tiles(ve))
    ve.close()


def test_bench_text_config_matches_oracle(bench_mod):
    import torch
    from open_clip_inference import _lib
    from open_clip_inference.engine import Engine
    B = bench_mod.B_TEXT
    dev = torch.device("cuda", 0)
    te = Engine(bench_mod.make_model_dir(), _lib.TOWER_TEXT, [0], "bf16", B)
    _, ids = bench_mod.synth_inputs(0, dev)
    out = torch.empty((B, 512), device=dev, dtype=torch.float32)
    s = torch.cuda.current_stream(dev)
    te.embed_tokens_device(ids.data_ptr(), B, out.data_ptr(), s.cuda_stream)
    torch.cuda.synchronize()
    first = out.cpu().numpy()
    te.embed_tokens_device(ids.data_ptr(), B, out.data_ptr(), s.cuda_stream)
    torch.cuda.synchronize()
    got = out.cpu().numpy()
    assert np.array_equal(first, got)
    assert np.all(np.abs(np.linalg.norm(got, axis=1) - 1) < 1e-5)
    t = text_spec_from_cfg(VIT_B_32_CFG["model_cfg"])
    ref = clip_ref.encode_text(weights.text_weights(t, 1234), t, ids[TEXT_ROWS].cpu().numpy())
    cos = clip_ref.cosine_rows(got[TEXT_ROWS], ref)
    print("bench text tiles", _tiles(te), "cos min", float(cos.min()))
    assert cos.min() >= COS_TOL, (cos.min(), _tiles(te))
    # the host entry point (trimming off: full-length rows) gives the same bits as the device one
    host = te.embed_tokens(ids[:64].cpu().numpy())
    assert np.array_equal(host, got[:64])
    te.close()


@pytest.mark.parametrize("tower", ["vision", "text"])
@pytest.mark.parametrize("which", ["default", "side", "null_array"])
@pytest.mark.parametrize("entry", ["plain", "gather"])
def test_device_entry_is_ordered_on_the_callers_stream(bench_mod, tower, which, entry):
    """include/clipgpu.h: the *_device entry points are stream-ordered on the caller's stream.
    The output is filled with NaN, the forward is enqueued, and a copy of the output is enqueued
    right behind it on the same stream with no synchronization in between: the copy must see the
    finished embeddings -- for torch's default (legacy null) stream and for a created stream, at
    the bench's batch (milliseconds of work, so a missing join would be caught).  The gathered
    entry points (one-rank communicator: the forward + the in-place all-gather) likewise, where a
    NULL entry -- or a NULL streams array ("null_array") -- is the legacy default stream too."""
    import torch
    from open_clip_inference import _lib
    from open_clip_inference.engine import Engine
    if which == "null_array" and entry == "plain":
        pytest.skip("a NULL streams array exists only on the gathered entry points")
    dev = torch.device("cuda", 0)
    px, ids = bench_mod.synth_inputs(0, dev)
    B = bench_mod.B_VISION if tower == "vision" else bench_mod.B_TEXT
    e = Engine(bench_mod.make_model_dir(), _lib.TOWER_VISION if tower == "vision" else _lib.TOWER_TEXT,
               [0], "bf16", B)
    if entry == "gather":
        e.comm_init_rank(Engine.comm_unique_id(), 1, 0)
    s = torch.cuda.current_stream(dev) if which != "side" else torch.cuda.Stream(dev)
    out = torch.empty((B, 512), device=dev, dtype=torch.float32)
    with torch.cuda.stream(s):
        for rep in range(3):  # capture, then replays of the graph
            out.fill_(float("nan"))
            if entry == "gather":
                gather = e.embed_pixels_gather_device if tower == "vision" else e.embed_tokens_gather_device
                gather([(px if tower == "vision" else ids).data_ptr()], [B], [out.data_ptr()],
                       None if which == "null_array" else [s.cuda_stream])
            elif tower == "vision":
                e.embed_pixels_device(px.data_ptr(), B, out.data_ptr(), s.cuda_stream)
            else:
                e.embed_tokens_device(ids.data_ptr(), B, out.data_ptr(), s.cuda_stream)
            snap = out.clone()
            s.synchronize()
            got = snap.cpu().numpy()
            assert not np.isnan(got).any(), (tower, which, rep)
            assert np.all(np.abs(np.linalg.norm(got, axis=1) - 1) < 1e-5)
    e.close()
