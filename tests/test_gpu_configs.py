"""BASELINE.json configs[3] and configs[4] at their per-GPU workloads (one MI355X).

configs[3]: ViT-SO400M-16-SigLIP2-384 vision, batch 1024 over 8 GPUs -> 128 images per GPU.
configs[4]: DFN5B-CLIP-ViT-H/14-378 vision + text, batch 512 over 8 GPUs -> 64 per GPU, with the
            fp8 MFMA weight path.

Each shard runs through the device entry point on an engine built as tools/bench_models.py builds
it (max_batch = the shard, the committed tile table), and is checked the way the reference's
per-batch contract reads (VisionEmbedder::embed_images / TextEmbedder::embed_texts return one
L2-normalised row per input, src/vision.rs:100-117, src/text.rs:148-169):
  - every row unit-norm;
  - sampled rows (first, second, middle, last) against the fp64 oracle on the same seeded weights
    (cosine >= 0.9999 for bf16; the fp8 bars of tests/test_gpu_mx.py for the lossy MX split);
  - the same rows bit-equal to a small-batch (B = 4) call of the same inputs on the same engine
    (a row never depends on the rest of its batch, the lane split or the tile rows per launch).
The multi-GPU part (8 ranks + the RCCL all-gather) is the driver's 8-GPU run.

Also here: SO400M at max_batch 1024 in ONE lane -- 589,824 token rows, whose c_proj A operand
(4352 columns) is past the 32-bit per-lane DMA offsets, so the GEMMs run as row chunks
(gemm.hip launch_gemm) -- bit-equal to small-batch calls.
"""
import numpy as np
import pytest

from oracle import clip_ref, weights
from oracle.model_spec import (OPENAI_MEAN, OPENAI_STD, SIGLIP_MEAN, SIGLIP_STD, SO400M_16_SIGLIP2_384_CFG,
                               VIT_H_14_378_CFG)
from tests.helpers import COS_TOL, make_model_dir, normalized_pixels, specs
from tests.test_gpu_mx import FP8_COS_TEXT, FP8_COS_VISION

pytestmark = pytest.mark.gpu

_ORACLE = {}


def _oracle_rows(cfg, tower, data, rows, key):
    """fp64 oracle embeddings of data[rows] (cached per input set)."""
    k = (key, tuple(rows))
    if k not in _ORACLE:
        v, t = specs(cfg)
        if tower == 0:
            _ORACLE[k] = clip_ref.encode_image(weights.vision_weights(v, 1234), v, data[rows])
        else:
            _ORACLE[k] = clip_ref.encode_text(weights.text_weights(t, 1234), t, data[rows])
    return _ORACLE[k]


def _device_embed(e, tower, data):
    import torch
    B = data.shape[0]
    x = torch.from_numpy(np.ascontiguousarray(data)).cuda()
    out = torch.empty((B, e.embed_dim), device="cuda", dtype=torch.float32)
    s = torch.cuda.current_stream()
    if tower == 0:
        e.embed_pixels_device(x.data_ptr(), B, out.data_ptr(), s.cuda_stream)
    else:
        e.embed_tokens_device(x.data_ptr(), B, out.data_ptr(), s.cuda_stream)
    torch.cuda.synchronize()
    return out.cpu().numpy()


def _shard(cfg, tower, B, seed):
    v, t = specs(cfg)
    if tower == 0:
        mean, std = (SIGLIP_MEAN, SIGLIP_STD) if cfg is SO400M_16_SIGLIP2_384_CFG else (OPENAI_MEAN, OPENAI_STD)
        return normalized_pixels(weights.synth_images_u8(seed, B, v.image_size), mean, std)
    return weights.synth_token_ids(seed, B, t.context_length, t.vocab_size, t.vocab_size - 2, t.vocab_size - 1,
                                   random_eot=True)


def _check_shard(cfg, tower, B, dtype, mx_sites, bar, label):
    from open_clip_inference.engine import Engine
    data = _shard(cfg, tower, B, 100 + B + tower)
    e = Engine(make_model_dir(cfg, 1234), tower, [0], dtype, B, mx_sites=mx_sites)
    got = _device_embed(e, tower, data)
    assert got.shape == (B, e.embed_dim)
    norms = np.linalg.norm(got.astype(np.float64), axis=1)
    assert np.all(np.abs(norms - 1) < 1e-5), norms
    rows = [0, 1, B // 2, B - 1]
    ref = _oracle_rows(cfg, tower, data, rows, (id(cfg), tower, B))
    cos = clip_ref.cosine_rows(got[rows], ref)
    print(f"\n[{label}] B={B} {dtype} {mx_sites or ''}: cos vs oracle {np.round(cos, 6).tolist()}")
    assert cos.min() >= bar, cos
    small = e.embed_pixels(data[rows]) if tower == 0 else e.embed_tokens(data[rows])
    assert np.array_equal(small, got[rows])
    e.close()


@pytest.mark.parametrize("dtype,mx_sites,bar", [("bf16", None, COS_TOL), ("fp8", None, FP8_COS_VISION)])
def test_so400m_siglip2_384_shard_128(dtype, mx_sites, bar):
    """configs[3]: the 128-image per-GPU shard of SO400M-16-SigLIP2-384 vision."""
    _check_shard(SO400M_16_SIGLIP2_384_CFG, 0, 128, dtype, mx_sites, bar, "SO400M vision")


def test_so400m_siglip2_text_shard_128():
    """The SigLIP2 text tower of the same model folder (the reference's README model,
    README.md:72-80; open_clip text_cfg no_causal_mask, pool_type "last", proj_bias): 27 layers of
    width 1152, 64-token context, 128 sequences per GPU, against the fp64 oracle (itself pinned to
    HF SiglipTextModel, tests/test_cpu_oracle.py)."""
    _check_shard(SO400M_16_SIGLIP2_384_CFG, 1, 128, "bf16", None, COS_TOL, "SO400M-SigLIP2 text")


# configs[4]: bf16; the shipped fp8 split (QKV, c_fc, c_proj in MX); and the split whose two towers
# both meet the north-star bar (vision MX at QKV only, text bf16 -- per-engine options).
@pytest.mark.parametrize("dtype,mx_sites,bar", [("bf16", None, COS_TOL), ("fp8", None, FP8_COS_VISION),
                                                ("fp8", "qkv", COS_TOL)])
def test_vit_h14_378_vision_shard_64(dtype, mx_sites, bar):
    _check_shard(VIT_H_14_378_CFG, 0, 64, dtype, mx_sites, bar, "ViT-H/14-378 vision")


@pytest.mark.parametrize("dtype,mx_sites,bar", [("bf16", None, COS_TOL), ("fp8", None, FP8_COS_TEXT)])
def test_vit_h14_text_shard_64(dtype, mx_sites, bar):
    _check_shard(VIT_H_14_378_CFG, 1, 64, dtype, mx_sites, bar, "ViT-H/14 text")


def test_h14_north_star_split_in_one_process():
    """configs[4] as one deployment that meets cos >= 0.9999 on both towers: an fp8 vision engine
    with MX at QKV only beside a bf16 text engine, both in this process (per-engine options, no
    process-wide environment)."""
    from open_clip_inference.engine import Engine
    d = make_model_dir(VIT_H_14_378_CFG, 1234)
    ve = Engine(d, 0, [0], "fp8", 4, mx_sites="qkv")
    fe = Engine(d, 0, [0], "fp8", 4)
    te = Engine(d, 1, [0], "bf16", 4)
    assert ve.info()[2] == ["qkv"] and fe.info()[2] == ["qkv", "fc", "proj"] and te.info()[2] == []
    px = _shard(VIT_H_14_378_CFG, 0, 2, 5)
    ids = _shard(VIT_H_14_378_CFG, 1, 3, 6)
    v = ve.embed_pixels(px)
    cos = clip_ref.cosine_rows(v, _oracle_rows(VIT_H_14_378_CFG, 0, px, [0, 1], "ns_v"))
    assert cos.min() >= COS_TOL, cos
    assert not np.array_equal(v, fe.embed_pixels(px))  # the two fp8 engines really differ
    ct = clip_ref.cosine_rows(te.embed_tokens(ids), _oracle_rows(VIT_H_14_378_CFG, 1, ids, [0, 1, 2], "ns_t"))
    assert ct.min() >= COS_TOL, ct


def test_so400m_max_batch_1024_one_lane_row_chunks():
    """SO400M at max_batch 1024 on one lane: 1024 x 576 token rows per GEMM launch, past the 32-bit
    DMA offsets for c_proj (589,824 x 4352 x 2 bytes > 2^31), so launch_gemm splits it into row
    chunks.  The batch is 8 copies of 128 images: every copy's rows equal each other and the
    small-batch call of the same images bit for bit, across the chunk boundaries."""
    from open_clip_inference.engine import Engine
    base = _shard(SO400M_16_SIGLIP2_384_CFG, 0, 128, 77)
    px = np.concatenate([base] * 8)
    e = Engine(make_model_dir(SO400M_16_SIGLIP2_384_CFG, 1234), 0, [0], "bf16", 1024, lanes=1)
    assert e.info()[1] == 1
    got = _device_embed(e, 0, px)
    assert np.all(np.abs(np.linalg.norm(got.astype(np.float64), axis=1) - 1) < 1e-5)
    for k in range(1, 8):
        assert np.array_equal(got[k * 128:(k + 1) * 128], got[:128]), k
    rows = [0, 63, 127]
    assert np.array_equal(e.embed_pixels(base[rows]), got[[1024 - 128 + r for r in rows]])
    cos = clip_ref.cosine_rows(got[[1023]], _oracle_rows(SO400M_16_SIGLIP2_384_CFG, 0, base, [127], "chunk"))
    assert cos.min() >= COS_TOL, cos
