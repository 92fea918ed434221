"""End-to-end through the drop-in API (open_clip_inference.{VisionEmbedder, TextEmbedder,
Clip}, mirror of src/vision.rs / src/text.rs / src/clip.rs) on the GPU: host
preprocessing + tokenizer (C++) + HIP towers, vs the oracle chain
(preprocess_ref -> clip_ref, tokenizer_ref -> clip_ref) at cosine >= 0.9999."""
import json
import os

import numpy as np
import pytest

from oracle import clip_ref, facade_ref, preprocess_ref, weights
from oracle.model_spec import OPENAI_MEAN, OPENAI_MODEL_CONFIG, OPENAI_STD, TINY_CFG, text_spec_from_cfg, \
    vision_spec_from_cfg
from oracle.tokenizer_ref import ClipTokenizerRef
from tests.helpers import COS_TOL, make_model_dir

pytestmark = pytest.mark.gpu

GOLD = os.path.join(os.path.dirname(__file__), "golden")
TOKJ = os.path.join(GOLD, "clip_synth_tokenizer.json")


def cfg_with_tokenizer(ctx=16):
    with open(TOKJ, encoding="utf-8") as f:
        tj = f.read()
    vocab = len(json.loads(tj)["model"]["vocab"])
    cfg = json.loads(json.dumps(TINY_CFG))
    cfg["model_cfg"]["text_cfg"]["vocab_size"] = vocab
    cfg["model_cfg"]["text_cfg"]["context_length"] = ctx
    mc = dict(OPENAI_MODEL_CONFIG, vocab_size=vocab)
    return cfg, tj, mc


@pytest.fixture(scope="module")
def model():
    cfg, tj, mc = cfg_with_tokenizer()
    d = make_model_dir(cfg, seed=77, tokenizer_json=tj, model_config=mc)
    return cfg, d


def images():
    g = np.load(os.path.join(GOLD, "preprocess_golden.npz"))
    ims = [g["cat_face_crop"], g["cat_face_224"]]
    ims += [weights.synth_images_u8(h * 1000 + w, 1, max(h, w))[0][:h, :w].copy()
            for h, w in ((389, 517), (97, 301))]
    return ims


def oracle_images(cfg, ims):
    v = vision_spec_from_cfg(cfg["model_cfg"])
    px = np.stack([preprocess_ref.preprocess(im, v.image_size, OPENAI_MEAN, OPENAI_STD) for im in ims])
    return clip_ref.encode_image(weights.vision_weights(v, 77), v, px)


def oracle_texts(cfg, texts):
    t = text_spec_from_cfg(cfg["model_cfg"])
    tok = ClipTokenizerRef(TOKJ, t.context_length, 0)
    ids = np.array([tok.encode(x)[0] for x in texts], np.int64)
    return clip_ref.encode_text(weights.text_weights(t, 77), t, ids)


TEXTS = ["A photo of a cat", "A photo of a dog", "A photo of a beignet", "Café naïve résumé", "",
         " ".join(["word"] * 40)]


def test_vision_embedder_end_to_end(model):
    from open_clip_inference import VisionEmbedder
    cfg, d = model
    ve = VisionEmbedder.from_local_dir(d).build()
    ims = images()
    got = ve.embed_images(ims)
    assert clip_ref.cosine_rows(got, oracle_images(cfg, ims)).min() >= COS_TOL
    one = ve.embed_image(ims[0])
    assert one.shape == (64,) and np.allclose(one, got[0], atol=1e-6)
    pre = ve.preprocess(ims[2])
    assert pre.shape == (1, 3, 64, 64)


def test_text_embedder_end_to_end(model):
    from open_clip_inference import TextEmbedder
    cfg, d = model
    te = TextEmbedder.from_local_dir(d).build()
    got = te.embed_texts(TEXTS)
    assert clip_ref.cosine_rows(got, oracle_texts(cfg, TEXTS)).min() >= COS_TOL
    ids, mask = te.tokenize(TEXTS)
    assert ids.shape == (len(TEXTS), 16) and mask.dtype == np.int64
    assert np.allclose(te.embed_text(TEXTS[1]), got[1], atol=1e-6)


def test_clip_facade_and_integration_shape(model):
    """tests/integration_test.rs:9-36 structure (classify cat_face against three labels); with
    synthetic weights the semantic assertion (p > 0.99) is replaced by agreement with the
    oracle facade on oracle embeddings."""
    from open_clip_inference import Clip
    cfg, d = model
    clip = Clip.from_local_dir(d).build()
    cat = images()[0]
    labels = TEXTS[:3]
    res = clip.classify(cat, labels)
    assert sorted(l for l, _ in res) == sorted(labels)
    assert abs(sum(p for _, p in res) - 1) < 1e-5
    assert all(res[i][1] >= res[i + 1][1] for i in range(len(res) - 1))
    ref = facade_ref.classify(oracle_images(cfg, [cat])[0], oracle_texts(cfg, labels), labels, 100.0, 0.0)
    # logit_scale 100 amplifies the <= 1e-4 cosine gap of each embedding: compare at 0.05
    assert np.allclose(sorted(p for _, p in res), sorted(p for _, p in ref), atol=0.05)
    ranks = clip.rank_images(images(), labels[0])
    assert sorted(i for i, _ in ranks) == [0, 1, 2, 3]
    assert isinstance(clip.compare(cat, labels[0]), float)
    assert clip.get_model_config().logit_scale == 100.0


def test_clip_classify_vit_b32_dims():
    """BASELINE configs[0] plumbing at the north-star model's dims (ViT-B/32-224 vision, 12 x 512
    text tower, 77-token context): Clip.classify(cat_face, three labels) as
    tests/integration_test.rs:16-29 calls it, against the oracle chain (preprocess_ref ->
    clip_ref, tokenizer_ref -> clip_ref -> facade_ref).  Seeded weights, so the semantic
    p > 0.99 assertion is replaced by agreement with the oracle facade."""
    from open_clip_inference import Clip
    from oracle.model_spec import VIT_B_32_CFG
    with open(TOKJ, encoding="utf-8") as f:
        tj = f.read()
    cfg = json.loads(json.dumps(VIT_B_32_CFG))
    d = make_model_dir(cfg, seed=1234, tokenizer_json=tj, model_config=OPENAI_MODEL_CONFIG)
    clip = Clip.from_local_dir(d).build()
    cat = images()[0]
    labels = ["A photo of a cat", "A photo of a dog", "A photo of a beignet"]
    res = clip.classify(cat, labels)
    v = vision_spec_from_cfg(cfg["model_cfg"])
    t = text_spec_from_cfg(cfg["model_cfg"])
    px = preprocess_ref.preprocess(cat, v.image_size, OPENAI_MEAN, OPENAI_STD)[None]
    img_ref = clip_ref.encode_image(weights.vision_weights(v, 1234), v, px)
    tok = ClipTokenizerRef(TOKJ, t.context_length, 0)
    ids = np.array([tok.encode(x)[0] for x in labels], np.int64)
    txt_ref = clip_ref.encode_text(weights.text_weights(t, 1234), t, ids)
    img = clip.vision.embed_image(cat)
    txt = clip.text.embed_texts(labels)
    assert clip_ref.cosine_rows(img[None], img_ref).min() >= COS_TOL
    assert clip_ref.cosine_rows(txt, txt_ref).min() >= COS_TOL
    ref = facade_ref.classify(img_ref[0], txt_ref, labels, 100.0, 0.0)
    assert sorted(l for l, _ in res) == sorted(labels)
    assert abs(sum(p for _, p in res) - 1) < 1e-5
    # logit_scale 100 amplifies the <= 1e-4 cosine gap of each embedding: compare at 0.05
    assert np.allclose([p for _, p in sorted(res)], [p for _, p in sorted(ref)], atol=0.05)
    # and the facade on the engine's own embeddings is the reference's arithmetic exactly
    exact = facade_ref.classify_f32_exact(img, txt, labels, 100.0, 0.0)
    assert [(l, np.float32(p)) for l, p in res] == [(l, np.float32(p)) for l, p in exact]


def test_duplicate_and_multi_replica_handle(model):
    """duplicate() gives an independent handle; a handle with devices [0, 0] exercises the
    multi-device row-sharding path (two replicas, two host workers) on one GPU."""
    from open_clip_inference import VisionEmbedder
    cfg, d = model
    ve = VisionEmbedder.from_local_dir(d).build()
    ims = images()
    a = ve.embed_images(ims)
    b = ve.duplicate().embed_images(ims)
    assert np.array_equal(a, b)
    multi = VisionEmbedder.from_local_dir(d).with_devices([0, 0]).with_max_batch(1).build()
    assert np.array_equal(multi.embed_images(ims), a)


def test_empty_batch_errors(model):
    from open_clip_inference import TextEmbedder, VisionEmbedder
    from open_clip_inference.error import InferenceError
    cfg, d = model
    with pytest.raises(InferenceError, match="Empty batch"):
        VisionEmbedder.from_local_dir(d).build().embed_images([])
    with pytest.raises(InferenceError, match="Empty batch"):
        TextEmbedder.from_local_dir(d).build().embed_texts([])


def resize_cases():
    rng = np.random.default_rng(5)
    sizes = [(389, 517), (97, 301), (224, 224), (2000, 1500), (64, 64), (33, 70), (1, 400), (700, 1),
             (500, 500), (81, 64)]
    return [rng.integers(0, 256, (h, w, 3), dtype=np.uint8) for h, w in sizes]


@pytest.mark.parametrize("interp,mode", [("bicubic", "shortest"), ("bilinear", "shortest"),
                                         ("nearest", "shortest"), ("bicubic", "squash"), ("bilinear", "squash")])
@pytest.mark.parametrize("size", [224, 64, 384])
def test_gpu_resize_bit_exact_vs_host(interp, mode, size):
    """a5 on the GPU (kernels/resize.hip, clipgpu_embed_images_rgb8's first step) == the host
    resize (pinned to the oracle / Pillow, test_cpu_preprocess.py) bit for bit: crop box,
    up- and down-scaling, identity sizes, 1-pixel-wide images."""
    from open_clip_inference.engine import resize_rgb8, resize_rgb8_gpu
    ims = resize_cases()
    got = resize_rgb8_gpu(ims, size, interp, mode)
    for i, im in enumerate(ims):
        ref = resize_rgb8(im, size, interp, mode)
        assert np.array_equal(got[i], ref), (i, im.shape, int(np.abs(got[i].astype(int) - ref).max()))


def test_embed_images_rgb8_matches_host_preprocess(model):
    """Decoded images -> embeddings with the crop/resize/normalise on the GPU: bit-identical to
    the host preprocess_batch + embed_pixels path, and at the oracle's cosine tolerance; a
    multi-replica handle shards them in input order."""
    from open_clip_inference import VisionEmbedder
    cfg, d = model
    ve = VisionEmbedder.from_local_dir(d).with_max_batch(4).build()
    ims = images() + resize_cases()[:6]
    host = ve.session.embed_pixels(ve.preprocess_batch(ims))
    gpu = ve.session.embed_images_rgb8(ims)
    assert np.array_equal(gpu, host)
    assert clip_ref.cosine_rows(gpu[:4], oracle_images(cfg, ims[:4])).min() >= COS_TOL
    multi = VisionEmbedder.from_local_dir(d).with_devices([0, 0]).with_max_batch(2).build()
    assert np.array_equal(multi.session.embed_images_rgb8(ims), gpu)


def test_embed_images_rgb8_identity_batches_take_the_u8_path():
    """A batch of image_size x image_size decoded images needs no resize (its plan is the identity), so
    clipgpu_embed_images_rgb8 sends it down the u8 host path (copy-pool staging, copy-stream H2Ds, two
    buffer sets past max_batch) instead of the resize kernels.  Bit-identical to the resize path
    (clipgpu_test_rgb8_resize_always) and to embed_u8 on the stacked images: one round, several rounds
    with a ragged last one, and a two-replica handle."""
    from oracle.model_spec import VIT_B_32_CFG
    from open_clip_inference import _lib
    from open_clip_inference.engine import Engine
    d = make_model_dir(VIT_B_32_CFG, seed=1234)
    v = vision_spec_from_cfg(VIT_B_32_CFG["model_cfg"])
    u8 = weights.synth_images_u8(83, 45, v.image_size)
    ims = [u8[i] for i in range(len(u8))]
    e = Engine(d, 0, [0], "bf16", 16)
    for n in (1, 16, 45):
        fast = e.embed_images_rgb8(ims[:n])
        _lib.check(_lib.lib().clipgpu_test_rgb8_resize_always(e.handle, 1))
        slow = e.embed_images_rgb8(ims[:n])
        _lib.check(_lib.lib().clipgpu_test_rgb8_resize_always(e.handle, 0))
        assert np.array_equal(fast, slow), n
        assert np.array_equal(fast, e.embed_u8(u8[:n], OPENAI_MEAN, OPENAI_STD)), n
    multi = Engine(d, 0, [0, 0], "bf16", 8)
    assert np.array_equal(multi.embed_images_rgb8(ims), e.embed_images_rgb8(ims))
    # a batch mixing sizes takes the resize path for every image: the S x S rows do not change
    mixed = ims[:3] + [np.ascontiguousarray(u8[3][:200])]
    assert np.array_equal(e.embed_images_rgb8(mixed)[:3], e.embed_images_rgb8(ims[:3]))
    e.close()
    multi.close()


@pytest.mark.parametrize("ni,nt,E", [(1, 3, 64), (300, 1000, 512), (1000, 1, 768), (65, 129, 1152), (7, 5000, 1024)])
@pytest.mark.parametrize("act,axis", [("softmax", 1), ("softmax", 0), ("sigmoid", 1), ("logits", 1)])
def test_similarity_kernel_vs_facade_math(ni, nt, E, act, axis):
    """The facade arithmetic on the device (kernels/similarity.hip) vs the restated
    src/clip.rs math in f64 (oracle/facade_ref.py): logits = dot * scale + bias; softmax along
    either axis / sigmoid.  Exact-f32 MFMA dot products: |err| <= 1e-5 relative."""
    from open_clip_inference.engine import similarity
    rng = np.random.default_rng(ni * 7 + nt + E)
    a = rng.standard_normal((ni, E)).astype(np.float32)
    a /= np.linalg.norm(a, axis=1, keepdims=True)
    b = rng.standard_normal((nt, E)).astype(np.float32)
    b /= np.linalg.norm(b, axis=1, keepdims=True)
    scale, bias = (100.0, 0.0) if act != "sigmoid" else (10.0, -10.0)
    got = similarity(a, b, scale, bias, act, axis)
    logits = a.astype(np.float64) @ b.T.astype(np.float64) * scale + bias
    if act == "logits":
        ref = logits
    elif act == "sigmoid":
        ref = facade_ref.sigmoid(logits)
    else:
        ref = np.apply_along_axis(facade_ref.softmax, axis, logits)
    tol = 2e-5 * np.abs(ref) + (3e-5 if act == "logits" else 1e-6)
    assert np.all(np.abs(got - ref) <= tol), float(np.abs(got - ref).max())


def test_classify_many_and_rank_images_many(model):
    """The batched facade (device math) agrees with the per-call facade on the same inputs."""
    from open_clip_inference import Clip
    cfg, d = model
    clip = Clip.from_local_dir(d).build()
    ims = images()
    labels = TEXTS[:4]
    many = clip.classify_many(ims, labels)
    assert len(many) == len(ims)
    for im, res in zip(ims, many):
        one = clip.classify(im, labels)
        assert [l for l, _ in res] == [l for l, _ in one] or np.allclose([p for _, p in res], [p for _, p in one],
                                                                         atol=1e-5)
        assert np.allclose(sorted(p for _, p in res), sorted(p for _, p in one), atol=1e-5)
    ranks = clip.rank_images_many(ims, labels[:2])
    for q, res in zip(labels[:2], ranks):
        one = clip.rank_images(ims, q)
        assert np.allclose(sorted(p for _, p in res), sorted(p for _, p in one), atol=1e-5)
        assert sorted(i for i, _ in res) == list(range(len(ims)))


def test_rccl_communicator_and_gathered_entry_points(monkeypatch):
    """The data-parallel collective inside the C ABI on a one-GPU box: a one-rank RCCL
    communicator (clipgpu_comm_unique_id + clipgpu_comm_init_rank, as each rank of a
    one-process-per-GPU deployment does), then the gathered entry points (forward of the rank's
    block + ncclAllGather, in place) equal the plain device forward bit for bit -- vision and
    text, a block larger than max_batch (chunked).  A handle listing one device twice has no
    communicator."""
    import torch
    from oracle.model_spec import VIT_B_32_CFG
    from open_clip_inference import _lib
    from open_clip_inference.engine import Engine
    from open_clip_inference.error import InferenceError
    from tests.helpers import normalized_pixels
    d = make_model_dir(VIT_B_32_CFG, seed=1234)
    v = vision_spec_from_cfg(VIT_B_32_CFG["model_cfg"])
    t = text_spec_from_cfg(VIT_B_32_CFG["model_cfg"])
    s = torch.cuda.current_stream()
    for tower in (0, 1):
        e = Engine(d, tower, [0], "bf16", 16)
        assert e.comm_info() == (0, 0)
        B = 40
        if tower == 0:
            x = normalized_pixels(weights.synth_images_u8(9, B, v.image_size), OPENAI_MEAN, OPENAI_STD)
        else:
            x = weights.synth_token_ids(9, B, t.context_length, t.vocab_size, t.vocab_size - 2, t.vocab_size - 1,
                                        random_eot=True)
        d_in = torch.from_numpy(x).cuda()
        out = torch.full((B, 512), float("nan"), device="cuda")
        gather = e.embed_pixels_gather_device if tower == 0 else e.embed_tokens_gather_device
        with pytest.raises(InferenceError, match="no communicator"):
            gather([d_in.data_ptr()], [B], [out.data_ptr()], [s.cuda_stream])
        e.comm_init_rank(Engine.comm_unique_id(), 1, 0)
        assert e.comm_info() == (1, 0)
        gather([d_in.data_ptr()], [B], [out.data_ptr()], [s.cuda_stream])
        torch.cuda.synchronize()
        got = out.cpu().numpy()
        ref = e.embed_pixels(x) if tower == 0 else e.embed_tokens(x)
        np.testing.assert_array_equal(got, ref, err_msg=f"tower {tower}")
        # the ragged branch (one ncclBroadcast per non-empty block, rank offsets) forced on the
        # equal one-rank block: the same bits
        _lib.check(_lib.lib().clipgpu_test_force_broadcast(e.handle, 1))
        out.fill_(float("nan"))
        gather([d_in.data_ptr()], [B], [out.data_ptr()], [s.cuda_stream])
        torch.cuda.synchronize()
        assert np.array_equal(out.cpu().numpy(), ref)
        _lib.check(_lib.lib().clipgpu_test_force_broadcast(e.handle, 0))
        e.close()
    multi = Engine(d, 0, [0, 0], "bf16", 4)
    assert multi.comm_info() == (0, 0)


def test_multi_round_host_calls_alternate_buffer_sets_bit_exactly():
    """A host-buffer call of more than max_batch rows runs its rounds on two alternating staging sets
    (engine.hip run_host_shard: round i + 1's H2D under round i's forward).  Every
    round must equal the same rows embedded by a call of their own, bit for bit: u8 and f32 pixels
    and token ids, pageable and caller-registered buffers, a ragged last round, and a second
    multi-round call (graph replay on both sets).  The staging copies run on the persistent copy pool
    in pieces, each piece's H2D issued as soon as it is packed."""
    import ctypes
    from oracle.model_spec import VIT_B_32_CFG
    from open_clip_inference import _lib
    from open_clip_inference.engine import Engine, host_register, host_unregister
    from tests.helpers import normalized_pixels
    d = make_model_dir(VIT_B_32_CFG, seed=1234)
    v = vision_spec_from_cfg(VIT_B_32_CFG["model_cfg"])
    t = text_spec_from_cfg(VIT_B_32_CFG["model_cfg"])
    MB, B = 16, 71  # 5 rounds, the last one of 7 rows
    u8 = weights.synth_images_u8(21, B, v.image_size)
    px = normalized_pixels(u8, OPENAI_MEAN, OPENAI_STD)
    ids = weights.synth_token_ids(21, B, t.context_length, t.vocab_size, t.vocab_size - 2, t.vocab_size - 1,
                                  random_eot=True)
    ve = Engine(d, 0, [0], "bf16", MB)
    te = Engine(d, 1, [0], "bf16", MB)
    calls = {"u8": (ve, lambda e, x, out=None: e.embed_u8(x, OPENAI_MEAN, OPENAI_STD, out=out), u8),
             "f32": (ve, lambda e, x, out=None: e.embed_pixels(x, out=out), px),
             "ids": (te, lambda e, x, out=None: e.embed_tokens(x, out=out), ids)}
    no_bounds = (ctypes.c_int * 4)()
    for name, (e, fn, x) in calls.items():
        ref = np.concatenate([fn(e, x[i:i + MB]) for i in range(0, B, MB)])
        for registered, flags in ((False, 1), (True, 1)):
            _lib.check(_lib.lib().clipgpu_test_host_plan(e.handle, 0, no_bounds, flags))
            from open_clip_inference.engine import host_buffer
            xin = host_buffer(x.shape, x.dtype)
            xin[...] = x
            out = host_buffer((B, 512), np.float32)
            if registered:
                host_register(xin)
                host_register(out)
            try:
                for _ in range(2):
                    out.fill(np.nan)
                    fn(e, xin, out=out)
                    assert np.array_equal(out, ref), (name, registered, flags)
            finally:
                if registered:
                    host_unregister(xin)
                    host_unregister(out)
    ve.close()
    te.close()


def test_one_device_clique_runs_the_multi_device_comm_path():
    """The multi-device handle's own communicator code on the one-GPU box: a
    one-device handle with clipgpu_options.communicator = 1 builds a one-rank clique through
    ensure_comm (ncclCommInitAll at creation), and one given the multi-device handle's lazy path
    (clipgpu_test_comm_lazy) builds it inside sharded_gather on its first gathered call.  The
    gathered calls equal the plain device entry point bit for bit; each handle is then destroyed
    while its last collective is still queued behind a busy caller stream (a created stream, and
    the legacy default stream through a NULL streams array): destroy_comms waits for
    the collective's event before the grouped ncclCommFinalize, so the output is complete."""
    import torch
    from oracle.model_spec import VIT_B_32_CFG
    from open_clip_inference import _lib
    from open_clip_inference.engine import Engine
    from tests.helpers import normalized_pixels
    d = make_model_dir(VIT_B_32_CFG, seed=1234)
    v = vision_spec_from_cfg(VIT_B_32_CFG["model_cfg"])
    t = text_spec_from_cfg(VIT_B_32_CFG["model_cfg"])
    B = 24
    for tower, lazy in ((0, False), (1, True), (0, True), (1, False)):
        if tower == 0:
            x = normalized_pixels(weights.synth_images_u8(13, B, v.image_size), OPENAI_MEAN, OPENAI_STD)
        else:
            x = weights.synth_token_ids(13, B, t.context_length, t.vocab_size, t.vocab_size - 2, t.vocab_size - 1,
                                        random_eot=True)
        plain = Engine(d, tower, [0], "bf16", 16)
        ref = plain.embed_pixels(x) if tower == 0 else plain.embed_tokens(x)
        plain.close()
        if lazy:
            e = Engine(d, tower, [0], "bf16", 16)
            assert e.comm_info() == (0, 0)
            _lib.check(_lib.lib().clipgpu_test_comm_lazy(e.handle))
        else:
            e = Engine(d, tower, [0], "bf16", 16, communicator=True)
        assert e.comm_info() == (1, 0)
        d_in = torch.from_numpy(x).cuda()
        gather = e.embed_pixels_gather_device if tower == 0 else e.embed_tokens_gather_device
        out = torch.full((B, 512), float("nan"), device="cuda")
        side = torch.cuda.Stream()
        gather([d_in.data_ptr()], [B], [out.data_ptr()], [side.cuda_stream])  # the lazy clique is built here
        side.synchronize()
        np.testing.assert_array_equal(out.cpu().numpy(), ref, err_msg=f"tower {tower} lazy {lazy}")
        # destroy with the collective still queued: behind ~50 ms of spinning on the caller's stream
        out2 = torch.full((B, 512), float("nan"), device="cuda")
        null_array = tower == 1
        busy = torch.cuda.default_stream() if null_array else side
        with torch.cuda.stream(busy):
            torch.cuda._sleep(100_000_000)
        gather([d_in.data_ptr()], [B], [out2.data_ptr()], None if null_array else [side.cuda_stream])
        e.close()
        torch.cuda.synchronize()
        assert np.array_equal(out2.cpu().numpy(), ref)


def test_tile_table_is_deterministic_and_bit_invisible():
    """The default tile choice is the committed table (engine.hip table_tiles): two engines of
    the bench's configuration pick the same tiles and lanes on any box (vision at 256 images: two
    lanes, qkv / c_fc / c_proj on the 4-wave 160x128 RS tile, out_proj on the 8-wave 224x192); a timing tuner
    (clipgpu_options.tuning) may pick others, with the same output bits."""
    from oracle.model_spec import VIT_B_32_CFG
    from open_clip_inference.engine import Engine
    from tests.helpers import normalized_pixels
    d = make_model_dir(VIT_B_32_CFG, seed=1234)
    a = Engine(d, 0, [0], "bf16", 256)
    b = Engine(d, 0, [0], "bf16", 256)
    assert a.info() == b.info() == ([15, 26, 15, 15], 2, [])
    t = Engine(d, 0, [0], "bf16", 256, tuning=True)
    v = vision_spec_from_cfg(VIT_B_32_CFG["model_cfg"])
    x = normalized_pixels(weights.synth_images_u8(31, 64, v.image_size), OPENAI_MEAN, OPENAI_STD)
    assert np.array_equal(a.embed_pixels(x), t.embed_pixels(x))
    # fp8 engines of the same configuration: the MX sites on the tuner's MX tiles (qkv 256x128, c_fc /
    # c_proj 128x128), out_proj on 160x128 RS
    f = Engine(d, 0, [0], "fp8", 256)
    assert f.info() == ([2, 15, 3, 3], 2, ["qkv", "fc", "proj"])
    f.close()
    small = Engine(d, 0, [0], "bf16", 8)  # rows < 2048: the shape heuristic
    assert small.info()[0] == [0, 0, 0, 0]
    # the text tower at the bench's 1024 x 77 batch: two lanes, c_proj on the 4-wave 160x128 RS
    # tile (table_lanes / table_tiles); same bits as a small engine on the heuristic tiles
    ta = Engine(d, 1, [0], "bf16", 1024)
    tb = Engine(d, 1, [0], "bf16", 1024)
    assert ta.info() == tb.info() == ([18, 17, 18, 15], 2, [])
    ts = Engine(d, 1, [0], "bf16", 8)
    rng = np.random.default_rng(5)
    ids = rng.integers(1, 49406, size=(8, 77)).astype(np.int64)
    ids[:, 0] = 49406
    ids[np.arange(8), rng.integers(5, 77, size=8)] = 49407
    assert np.array_equal(ta.embed_tokens(ids), ts.embed_tokens(ids))


def test_siglip2_text_embedder_and_clip_end_to_end():
    """The reference's README model family (README.md:72-80, timm/ViT-SO400M-16-SigLIP2-384):
    a SigLIP2-structured folder -- SigLIP vision + SigLIP2 text tower (no causal mask, last-position
    pooling, projection bias), a Gemma-structured tokenizer.json (SentencePiece BPE with byte
    fallback, tests/golden/gemma_synth_tokenizer.json) and pull_onnx.py:140-150's SigLIP2
    model_config (sigmoid, lowercase, pad id 0) -- through TextEmbedder and Clip, against the
    tokenizers wheel + fp64 oracle chain."""
    tokenizers = pytest.importorskip("tokenizers")
    from oracle.model_spec import SIGLIP_MEAN, SIGLIP_STD, tiny_siglip_cfg
    from open_clip_inference import Clip, TextEmbedder
    path = os.path.join(GOLD, "gemma_synth_tokenizer.json")
    with open(path, encoding="utf-8") as f:
        tj = f.read()
    vocab = len(json.loads(tj)["model"]["vocab"])
    cfg = tiny_siglip_cfg()
    cfg["model_cfg"]["text_cfg"]["vocab_size"] = vocab
    mc = {"logit_scale": 10.0, "logit_bias": -10.0, "activation_function": "sigmoid",
          "tokenizer_needs_lowercase": True, "pad_id": 0, "vocab_size": vocab}
    d = make_model_dir(cfg, seed=78, tokenizer_json=tj, model_config=mc)
    t = text_spec_from_cfg(cfg["model_cfg"])
    ref_tok = tokenizers.Tokenizer.from_file(path)
    ref_tok.enable_padding(length=t.context_length, pad_id=0)
    ref_tok.enable_truncation(max_length=t.context_length)
    ids = np.array([e.ids for e in ref_tok.encode_batch([x.lower() for x in TEXTS])], np.int64)
    want = clip_ref.encode_text(weights.text_weights(t, 78), t, ids)
    te = TextEmbedder.from_local_dir(d).build()
    got_ids, _ = te.tokenize(TEXTS)
    assert np.array_equal(got_ids, ids)
    got = te.embed_texts(TEXTS)
    assert clip_ref.cosine_rows(got, want).min() >= COS_TOL
    clip = Clip.from_local_dir(d).build()
    v = vision_spec_from_cfg(cfg["model_cfg"])
    px = np.stack([preprocess_ref.preprocess(im, v.image_size, SIGLIP_MEAN, SIGLIP_STD, mode="shortest")
                   for im in images()[:1]])
    img = clip_ref.encode_image(weights.vision_weights(v, 78), v, px)[0]
    res = clip.classify(images()[0], TEXTS[:3])
    ref = facade_ref.classify(img, want[:3], TEXTS[:3], 10.0, -10.0, activation="sigmoid")
    assert np.allclose(sorted(p for _, p in res), sorted(p for _, p in ref), atol=0.02)
