"""Per-kernel numerics on the GPU vs numpy references of the same op.

Every kernel of the hot path runs in isolation through include/clipgpu_testing.h
hooks; inputs are pre-rounded to the kernel's 16-bit operand type so that the
comparison isolates accumulation/epilogue error.  Tolerances are stated per test.
"""
import numpy as np
import pytest

from oracle import clip_ref

pytestmark = pytest.mark.gpu

BF16, F16 = 0, 1


def _lib():
    from open_clip_inference import _lib
    return _lib


def round16(x, dtype):
    x = np.asarray(x, np.float32)
    if dtype == F16:
        return x.astype(np.float16).astype(np.float32)
    u = x.view(np.uint32).astype(np.uint64)
    u = ((u + 0x7FFF + ((u >> 16) & 1)) & 0xFFFF0000).astype(np.uint32)
    return u.view(np.float32)


def ref_act(act, x):
    return {0: lambda v: v, 1: lambda v: clip_ref.act_fn("quick_gelu", v),
            2: lambda v: clip_ref.act_fn("gelu", v), 3: lambda v: clip_ref.act_fn("gelu_tanh", v)}[act](x)


def run_gemm(dtype, mode, act, A, W, bias=None, resid=None):
    L = _lib()
    M, K = A.shape
    N = W.shape[0]
    out = np.empty((M, N), np.float32)
    A = np.ascontiguousarray(A, np.float32)
    W = np.ascontiguousarray(W, np.float32)
    b = None if bias is None else np.ascontiguousarray(bias, np.float32)
    r = None if resid is None else np.ascontiguousarray(resid, np.float32)
    L.check(L.lib().clipgpu_test_gemm(dtype, mode, act, M, N, K, A.ctypes.data, W.ctypes.data,
                                      None if b is None else b.ctypes.data,
                                      None if r is None else r.ctypes.data, out.ctypes.data))
    return out


# every GEMM tile the library builds (kernels.hpp kGemmTiles; test_cpu_abi checks this list against it)
BUILT_TILES = [2, 3, 13, 14, 15, 17, 18, 26]


@pytest.fixture(params=BUILT_TILES,
                ids=["pipe256x128", "pipe256x256", "w8_192x256", "rs_256x256", "rs_160x128",
                     "rs_w8_160x128", "half_256x256", "w8_224x192"])
def tile(request, monkeypatch):
    """Every GEMM tile configuration (GemmTile) through the same numerics checks."""
    monkeypatch.setenv("CLIPGPU_TEST_TILE", str(request.param))
    return request.param


@pytest.mark.parametrize("dtype", [BF16, F16])
@pytest.mark.parametrize("M,N,K", [(128, 128, 64), (200, 136, 192), (1000, 768, 768), (77, 64, 512),
                                   (12800, 768, 3072), (2600, 3072, 768), (3000, 520, 384)])
def test_gemm_f32_out(dtype, M, N, K, tile):
    rng = np.random.default_rng(M * 7 + N + K)
    A = round16(rng.standard_normal((M, K)), dtype)
    W = round16(rng.standard_normal((N, K)) / np.sqrt(K), dtype)
    bias = rng.standard_normal(N).astype(np.float32)
    out = run_gemm(dtype, 2, 0, A, W, bias)
    ref = A.astype(np.float64) @ W.T.astype(np.float64) + bias
    # f32 accumulation of exact 16-bit products: |err| <~ 1e-6 * sum|a*b|
    bound = 3e-5 * (np.abs(A) @ np.abs(W).T) + 1e-6
    assert np.all(np.abs(out - ref) <= bound)


@pytest.mark.parametrize("dtype", [BF16, F16])
@pytest.mark.parametrize("act", [0, 1, 2, 3])
def test_gemm_store16_act(dtype, act, tile):
    M, N, K = 600, 384, 256
    rng = np.random.default_rng(act)
    A = round16(rng.standard_normal((M, K)), dtype)
    W = round16(rng.standard_normal((N, K)) / np.sqrt(K), dtype)
    bias = rng.standard_normal(N).astype(np.float32)
    out = run_gemm(dtype, 0, act, A, W, bias)
    ref = ref_act(act, A.astype(np.float64) @ W.T.astype(np.float64) + bias)
    rel = 2 ** -8 if dtype == BF16 else 2 ** -11  # one 16-bit output rounding (+ slack)
    assert np.all(np.abs(out - ref) <= 1.01 * rel * np.abs(ref) + 1e-4)


@pytest.mark.parametrize("dtype", [BF16])
def test_gemm_residual(dtype, tile):
    M, N, K = 1513, 640, 256
    rng = np.random.default_rng(5)
    A = round16(rng.standard_normal((M, K)), dtype)
    W = round16(rng.standard_normal((N, K)) / np.sqrt(K), dtype)
    bias = rng.standard_normal(N).astype(np.float32)
    resid = rng.standard_normal((M, N)).astype(np.float32)
    out = run_gemm(dtype, 1, 0, A, W, bias, resid)
    ref = resid + A.astype(np.float64) @ W.T.astype(np.float64) + bias
    assert np.abs(out - ref).max() < 1e-4


def _poison_lib():
    """lib/libclipgpu_poison.so (Makefile `poison`, built by `all`): the product library with the
    pipelined GEMM's LDS-DMA destinations NaN-filled before every DMA."""
    import ctypes
    import os
    path = os.environ.get("CLIPGPU_POISON_LIB") or os.path.join(
        os.path.dirname(os.path.abspath(__file__)), "..", "clip-embedder-rs_amd", "lib", "libclipgpu_poison.so")
    if not os.path.exists(path):
        pytest.skip("race-check library not built (make -C clip-embedder-rs_amd poison)")
    L = ctypes.CDLL(path)
    L.clipgpu_test_gemm.argtypes = [ctypes.c_int] * 3 + [ctypes.c_int64] * 3 + [ctypes.c_void_p] * 5
    L.clipgpu_test_gemm.restype = ctypes.c_int
    L.clipgpu_last_error.restype = ctypes.c_char_p
    return L


@pytest.mark.parametrize("M,N,K,mode,act", [(12800, 3072, 768, 0, 1), (6400, 3072, 768, 0, 1), (6400, 3072, 768, 2, 0),
                                            (12801, 3072, 768, 0, 1), (12800, 3072, 768, 1, 0)])
def test_half_tile_last_round_is_bit_exact(M, N, K, mode, act, monkeypatch):
    """TILE_256x256_HALF (18) at shapes where its half-tile last round applies (256 CUs: 600 / 300 /
    650 tiles of 256x256 leave a partial round of <= 16 tiles per XCD): bit-equal to the plain
    256x256 RS tile, and the race-check build (NaN-poisoned LDS-DMA destinations) too."""
    rng = np.random.default_rng(M + N)
    A = np.ascontiguousarray(round16(rng.standard_normal((M, K)), BF16))
    W = np.ascontiguousarray(round16(rng.standard_normal((N, K)) / np.sqrt(K), BF16))
    bias = rng.standard_normal(N).astype(np.float32)
    monkeypatch.setenv("CLIPGPU_TEST_TILE", "14")
    want = run_gemm(BF16, mode, act, A, W, bias)
    monkeypatch.setenv("CLIPGPU_TEST_TILE", "18")
    assert np.array_equal(run_gemm(BF16, mode, act, A, W, bias), want)
    P = _poison_lib()
    got = np.empty((M, N), np.float32)
    rc = P.clipgpu_test_gemm(BF16, mode, act, M, N, K, A.ctypes.data, W.ctypes.data, bias.ctypes.data, None,
                             got.ctypes.data)
    assert rc == 0, P.clipgpu_last_error()
    assert np.array_equal(got, want), int(np.isnan(got).sum())


@pytest.mark.parametrize("M,N,K,mode,act", [(1000, 768, 3072, 1, 0), (2600, 3072, 768, 0, 1), (333, 520, 1280, 2, 0),
                                            (6400, 768, 3072, 1, 0)])
def test_gemm_pipelines_never_read_a_stage_before_its_dma_lands(M, N, K, mode, act, monkeypatch):
    """Race check of the LDS-DMA schedules (2- and 3-stage, every pipelined tile, persistent
    multi-tile walks, M / N tails): in the poison build every DMA destination holds NaN until the
    DMA lands, so a fragment or bias read that runs ahead of its vmcnt wait / barrier turns the
    output NaN.  The outputs must equal the product build's bit for bit.  (The 3-stage schedule
    runs on the 224x192 tile at K >= 192.)"""
    P = _poison_lib()
    rng = np.random.default_rng(M + N + K)
    A = np.ascontiguousarray(round16(rng.standard_normal((M, K)), BF16))
    W = np.ascontiguousarray(round16(rng.standard_normal((N, K)) / np.sqrt(K), BF16))
    bias = rng.standard_normal(N).astype(np.float32)
    resid = rng.standard_normal((M, N)).astype(np.float32) if mode == 1 else None
    for t in BUILT_TILES[1:]:
        monkeypatch.setenv("CLIPGPU_TEST_TILE", str(t))
        want = run_gemm(BF16, mode, act, A, W, bias, resid)
        got = np.empty((M, N), np.float32)
        rc = P.clipgpu_test_gemm(BF16, mode, act, M, N, K, A.ctypes.data, W.ctypes.data, bias.ctypes.data,
                                 None if resid is None else resid.ctypes.data, got.ctypes.data)
        assert rc == 0, P.clipgpu_last_error()
        assert np.array_equal(got, want), (t, int(np.isnan(got).sum()))


@pytest.mark.parametrize("M,N,K,mode", [(12800, 768, 3072, 1), (12800, 768, 768, 1), (12801, 776, 3072, 1),
                                        (1000, 768, 128, 1), (6400, 768, 3072, 2), (12800, 3072, 768, 0),
                                        (6400, 768, 3072, 3), (6400, 768, 768, 3), (20000, 768, 768, 3),
                                        (12801, 776, 3072, 3), (1000, 768, 320, 3), (1000, 768, 256, 3)])
def test_224x192_residual_tile_is_bit_exact(M, N, K, mode, monkeypatch):
    """TILE_224x192_W8 (26: 3 LDS stages with an uneven DMA piece split, 52 pieces over 8 waves, so
    per-wave counted waits) with the NI = 3 column permutation and W swizzle
    (tools/lds_swizzle_check.py).  Bit-equal
    to the table's 160x128 tile 17 at the ViT-B/32 residual shapes (one round of 232 tiles), with M / N
    tails, 2 K-steps (the 2-stage fallback), and a persistent multi-tile walk through the 3-stage
    pipeline with the 16-bit QuickGELU epilogue (12800 x 3072: 928 tiles over 256 blocks); the race-check
    build gives the same bits.  Mode 3: the f16 residual stream (the engines' default) at the lane shapes
    of out_proj / c_proj (one tile per block), a persistent walk (20000 rows: 360 tiles over 256 blocks),
    M / N tails and short K."""
    rng = np.random.default_rng(M + N + K + mode)
    A = np.ascontiguousarray(round16(rng.standard_normal((M, K)), BF16))
    W = np.ascontiguousarray(round16(rng.standard_normal((N, K)) / np.sqrt(K), BF16))
    bias = rng.standard_normal(N).astype(np.float32)
    resid = rng.standard_normal((M, N)).astype(np.float32) if mode in (1, 3) else None
    act = 1 if mode == 0 else 0
    monkeypatch.setenv("CLIPGPU_TEST_TILE", "17")
    want = run_gemm(BF16, mode, act, A, W, bias, resid)
    P = _poison_lib()
    for t in ("26",):
        monkeypatch.setenv("CLIPGPU_TEST_TILE", t)
        assert np.array_equal(run_gemm(BF16, mode, act, A, W, bias, resid), want), t
        got = np.empty((M, N), np.float32)
        rc = P.clipgpu_test_gemm(BF16, mode, act, M, N, K, A.ctypes.data, W.ctypes.data, bias.ctypes.data,
                                 None if resid is None else resid.ctypes.data, got.ctypes.data)
        assert rc == 0, P.clipgpu_last_error()
        assert np.array_equal(got, want), (t, int(np.isnan(got).sum()))


@pytest.mark.parametrize("mode,act", [(0, 1), (0, 2), (1, 0), (2, 0)])
@pytest.mark.parametrize("M,N,K", [(1, 512, 768), (5, 64, 256), (77, 768, 768), (128, 3072, 768),
                                   (128, 768, 3072), (200, 2304, 1024), (256, 512, 768)])
def test_skinny_gemm_is_bit_exact(mode, act, M, N, K, monkeypatch):
    """The skinny kernel (TILE_AUTO's pick at M <= 256: the pruned last layer and the heads)
    gives the same bits as the tiled kernels: same MFMA operand roles, k -> lane assignment
    and K order, same epilogue float ops.  Also within the f32-accumulation bound of fp64."""
    rng = np.random.default_rng(M * 13 + N + K + mode)
    A = round16(rng.standard_normal((M, K)), BF16)
    W = round16(rng.standard_normal((N, K)) / np.sqrt(K), BF16)
    bias = rng.standard_normal(N).astype(np.float32)
    resid = rng.standard_normal((M, N)).astype(np.float32) if mode == 1 else None
    outs = []
    for t in ["100", "15", "14", "101"]:
        monkeypatch.setenv("CLIPGPU_TEST_TILE", t)
        outs.append(run_gemm(BF16, mode, act, A, W, bias, resid))
    assert all(np.array_equal(outs[0], o) for o in outs[1:])
    if mode == 2:
        ref = A.astype(np.float64) @ W.T.astype(np.float64) + bias
        assert np.all(np.abs(outs[0] - ref) <= 3e-5 * (np.abs(A) @ np.abs(W).T) + 1e-6)


@pytest.mark.parametrize("M", [800, 3000])
@pytest.mark.parametrize("mode,act", [(0, 1), (1, 0), (2, 0), (3, 0)])
def test_general_gemm_is_bit_exact(M, mode, act, monkeypatch):
    """The skinny kernel's general form (TILE_GENERAL 101: any M, N tails, element stores) -- what
    runs the shapes the pipelined tiles do not take since round 6 removed the 128x128 bt kernel --
    gives the pipelined tiles' bits at M = 800 and 3000 for every epilogue: the 16-bit store with an
    activation, the f32 and the f16 residual stream (modes 1 / 3) and the f32 store.  Then the shapes
    only it takes: K = 64 at any M, and a 16-bit output row of 100 elements (not a multiple of 8),
    within the f32-accumulation bound of fp64, with N tails."""
    rng = np.random.default_rng(M + mode)
    N, K = 520, 384
    A = round16(rng.standard_normal((M, K)), BF16)
    W = round16(rng.standard_normal((N, K)) / np.sqrt(K), BF16)
    bias = rng.standard_normal(N).astype(np.float32)
    resid = (rng.standard_normal((M, N)) * 30).astype(np.float32) if mode in (1, 3) else None
    outs = {}
    for t in ["101", "15", "14", "26"]:
        monkeypatch.setenv("CLIPGPU_TEST_TILE", t)
        outs[t] = run_gemm(BF16, mode, act, A, W, bias, resid)
    for t in ("15", "14", "26"):
        assert np.array_equal(outs[t], outs["101"]), t
    monkeypatch.setenv("CLIPGPU_TEST_TILE", "0")
    for n, k in [(136, 64), (100, 256), (100, 64), (40, 64)]:
        A2, W2 = A[:, :k], round16(rng.standard_normal((n, k)) / np.sqrt(k), BF16)
        b2 = bias[:n]
        r2 = None if resid is None else np.ascontiguousarray(resid[:, :n])
        got = run_gemm(BF16, mode, act, A2, W2, b2, r2)
        ref = A2.astype(np.float64) @ W2.T.astype(np.float64) + b2
        if mode == 0:
            ref = ref_act(act, ref)
            assert np.all(np.abs(got - ref) <= 1.01 * 2 ** -8 * np.abs(ref) + 1e-4), (n, k)
        elif mode == 2:
            assert np.all(np.abs(got - ref) <= 3e-5 * (np.abs(A2) @ np.abs(W2).T) + 1e-6), (n, k)
        else:
            r16 = r2 if mode == 1 else r2.astype(np.float16).astype(np.float64)
            tol = 1e-4 if mode == 1 else 2 ** -11 * np.abs(ref + r16) + 1e-3
            assert np.all(np.abs(got - (ref + r16)) <= tol), (n, k)


@pytest.mark.parametrize("mode", [0, 1])
def test_gemm_persistent_multi_tile(mode, tile):
    """ntiles > grid for every tile config (each block walks >= 2 tiles, the pipelined
    kernels' DMA cursor crosses tile boundaries), with M and N tails."""
    dtype = BF16
    M, N, K = 8300, 2056, 128
    rng = np.random.default_rng(11 + mode)
    A = round16(rng.standard_normal((M, K)), dtype)
    W = round16(rng.standard_normal((N, K)) / np.sqrt(K), dtype)
    bias = rng.standard_normal(N).astype(np.float32)
    if mode == 0:
        out = run_gemm(dtype, 0, 1, A, W, bias)
        ref = ref_act(1, A.astype(np.float64) @ W.T.astype(np.float64) + bias)
        assert np.all(np.abs(out - ref) <= 1.01 * 2 ** -8 * np.abs(ref) + 1e-4)
    else:
        resid = rng.standard_normal((M, N)).astype(np.float32)
        out = run_gemm(dtype, 1, 0, A, W, bias, resid)
        ref = resid + A.astype(np.float64) @ W.T.astype(np.float64) + bias
        assert np.abs(out - ref).max() < 1e-4


def run_lnf(dtype, act, x, wf, cs, bias, eps, tile, lib=None):
    """clipgpu_test_gemm_lnf (EPI_LNF): x / wf rounded to f16 on upload, output widened to f32."""
    M, K = x.shape
    N = wf.shape[0]
    out = np.empty((M, N), np.float32)
    args = [np.ascontiguousarray(a, np.float32) for a in (x, wf, cs, bias)]
    if lib is None:
        L = _lib()
        L.check(L.lib().clipgpu_test_gemm_lnf(dtype, act, M, N, K, *[a.ctypes.data for a in args], eps, tile,
                                              out.ctypes.data))
    else:
        import ctypes
        f = lib.clipgpu_test_gemm_lnf
        f.argtypes = [ctypes.c_int, ctypes.c_int] + [ctypes.c_int64] * 3 + [ctypes.c_void_p] * 4 + \
            [ctypes.c_float, ctypes.c_int, ctypes.c_void_p]
        f.restype = ctypes.c_int
        rc = f(dtype, act, M, N, K, *[a.ctypes.data for a in args], eps, tile, out.ctypes.data)
        assert rc == 0, lib.clipgpu_last_error()
    return out


def lnf_case(M, N, K, seed):
    """A residual-stream-like x (f16: per-row offsets, a few large channels), a Linear behind a
    LayerNorm (gamma, beta), and its fold: W' = f16(W diag(gamma)), cs = row sums of W', bias b + W beta."""
    rng = np.random.default_rng(seed)
    x = rng.standard_normal((M, K)) * rng.uniform(0.5, 4.0, (M, 1)) + rng.standard_normal((M, 1))
    x[:, rng.choice(K, 3, replace=False)] *= 40.0  # the stream's massive channels
    x = x.astype(np.float16).astype(np.float64)
    w = rng.standard_normal((N, K)) / np.sqrt(K)
    gamma = 1.0 + 0.2 * rng.standard_normal(K)
    beta = 0.1 * rng.standard_normal(K)
    b = 0.1 * rng.standard_normal(N)
    wf = (w.astype(np.float32) * gamma.astype(np.float32)).astype(np.float16).astype(np.float64)
    cs = wf.sum(1)
    bp = b + w.astype(np.float32).astype(np.float64) @ beta.astype(np.float32).astype(np.float64)
    return x, w, gamma, beta, b, wf, cs, bp


@pytest.mark.parametrize("M,N,K,act", [(77, 2304, 768, 0), (250, 3072, 768, 1), (3000, 2304, 768, 0),
                                       (6400, 3072, 768, 1), (12801, 1536, 512, 0), (1000, 2048, 512, 2)])
def test_layernorm_folded_gemm(M, N, K, act):
    """EPI_LNF (ln_1 / ln_2 folded into QKV / c_fc): every tile -- and the skinny kernel at M <= 256 --
    gives the same bits (each row's (mean, rstd) come from the statistics pass, launch_ln_stats, and
    every tile runs the same K-ordered MFMA chain and epilogue ops), and the result matches
    LayerNorm-then-Linear in fp64 within the bf16 output rounding plus the f16 rounding of
    W diag(gamma) (|err| <= 2^-7 |ref| + 0.01 rms(ref))."""
    x, w, gamma, beta, b, wf, cs, bp = lnf_case(M, N, K, M + N + act)
    eps = 1e-5
    tiles = [0] + BUILT_TILES + ([100] if M <= 256 else [])
    outs = [run_lnf(BF16, act, x, wf, cs, bp, eps, t) for t in tiles]
    for t, o in zip(tiles[1:], outs[1:]):
        assert np.array_equal(o, outs[0]), t
    mu = x.mean(1, keepdims=True)
    var = ((x - mu) ** 2).mean(1, keepdims=True)
    ref = ref_act(act, ((x - mu) / np.sqrt(var + eps) * gamma + beta) @ w.T + b)
    err = np.abs(outs[0] - ref)
    assert np.all(err <= 2 ** -7 * np.abs(ref) + 0.01 * np.sqrt(np.mean(ref ** 2))), float(err.max())
    # f16 output (f16 engines): the same sums, rounded to f16
    o16 = run_lnf(F16, act, x, wf, cs, bp, eps, 0)
    assert np.all(np.abs(o16 - ref) <= 2 ** -9 * np.abs(ref) + 0.01 * np.sqrt(np.mean(ref ** 2)))
    if M == 6400:  # race check: the column-sum DMA beside the bias DMA, every pipelined tile
        P = _poison_lib()
        for t in BUILT_TILES[1:]:
            assert np.array_equal(run_lnf(BF16, act, x, wf, cs, bp, eps, t, lib=P), outs[0]), t


def ref_attention(qkv, B, N, H, causal, HD=64):
    D = H * HD
    x = qkv.reshape(B, N, 3, H, HD).astype(np.float64)
    q, k, v = x[:, :, 0].transpose(0, 2, 1, 3), x[:, :, 1].transpose(0, 2, 1, 3), x[:, :, 2].transpose(0, 2, 1, 3)
    s = q @ k.transpose(0, 1, 3, 2) / np.sqrt(HD)
    if causal:
        s = np.where(np.triu(np.ones((N, N), bool), 1), -np.inf, s)
    o = clip_ref.softmax(s) @ v
    return o.transpose(0, 2, 1, 3).reshape(B * N, D)


@pytest.mark.parametrize("dtype", [BF16, F16])
@pytest.mark.parametrize("B,N,H,causal", [(3, 50, 12, 0), (4, 77, 8, 1), (2, 17, 2, 0), (2, 100, 2, 1),
                                          (1, 256, 2, 0), (2, 1, 2, 1)])
def test_attention(dtype, B, N, H, causal):
    L = _lib()
    rng = np.random.default_rng(N + H)
    qkv = round16(rng.standard_normal((B * N, 3 * H * 64)) * 1.5, dtype)
    out = np.empty((B * N, H * 64), np.float32)
    L.check(L.lib().clipgpu_test_attention(dtype, B, N, H, 64, causal, qkv.ctypes.data, out.ctypes.data))
    ref = ref_attention(qkv, B, N, H, causal)
    # P and O are rounded to 16 bits: |err| <= ~2 ulp16 of max|v|
    tol = (2 ** -7 if dtype == BF16 else 2 ** -10) * np.abs(qkv).max()
    assert np.abs(out - ref).max() < tol


@pytest.mark.parametrize("dtype", [BF16, F16])
@pytest.mark.parametrize("B,N,H,causal", [(300, 50, 12, 0), (700, 77, 8, 1), (1500, 9, 3, 1)])
def test_attention_large_batch(dtype, B, N, H, causal):
    """Bench-sized short-sequence launches (thousands of (sequence, head) workgroups, several
    rounds over the CUs): checked against the float64 reference, and bit for bit against calls on
    3-sequence slices at the start, middle and end of the batch (a sequence's result must not
    depend on the batch around it; profiles/r03_v11_attn_persistent_ab.txt ran this test against
    a persistent prefetching variant of the kernel as well)."""
    L = _lib()
    rng = np.random.default_rng(B + N)
    D = H * 64
    qkv = round16(rng.standard_normal((B * N, 3 * D)) * 1.5, dtype)
    out = np.empty((B * N, D), np.float32)
    L.check(L.lib().clipgpu_test_attention(dtype, B, N, H, 64, causal, qkv.ctypes.data, out.ctypes.data))
    ref = ref_attention(qkv, B, N, H, causal)
    tol = (2 ** -7 if dtype == BF16 else 2 ** -10) * np.abs(qkv).max()
    assert np.abs(out - ref).max() < tol
    for s0 in (0, B // 2, B - 3):
        sub = np.ascontiguousarray(qkv[s0 * N:(s0 + 3) * N])
        o3 = np.empty((3 * N, D), np.float32)
        L.check(L.lib().clipgpu_test_attention(dtype, 3, N, H, 64, causal, sub.ctypes.data, o3.ctypes.data))
        assert np.array_equal(o3, out[s0 * N:(s0 + 3) * N]), s0


@pytest.mark.parametrize("dtype", [BF16, F16])
@pytest.mark.parametrize("B,N,H,HD,causal", [(2, 300, 2, 64, 0), (2, 300, 2, 64, 1), (2, 577, 2, 72, 0),
                                             (2, 730, 2, 80, 0), (3, 130, 3, 80, 1), (2, 64, 1, 72, 0),
                                             (1, 1025, 1, 64, 1)])
def test_attention_tiled(dtype, B, N, H, HD, causal):
    """Tiled online-softmax kernel: long sequences (SigLIP2-384 576 tokens, ViT-H/14-378 730) and
    head dims 72 / 80 (scale 1/sqrt(HD)), partial last key/query tiles, causal masks."""
    L = _lib()
    rng = np.random.default_rng(N * 3 + HD + causal)
    D = H * HD
    qkv = round16(rng.standard_normal((B * N, 3 * D)), dtype)
    out = np.empty((B * N, D), np.float32)
    L.check(L.lib().clipgpu_test_attention(dtype, B, N, H, HD, causal, qkv.ctypes.data, out.ctypes.data))
    ref = ref_attention(qkv, B, N, H, causal, HD)
    tol = (2 ** -7 if dtype == BF16 else 2 ** -10) * np.abs(qkv).max()
    assert np.abs(out - ref).max() < tol


@pytest.mark.parametrize("dtype", [BF16, F16])
@pytest.mark.parametrize("D", [128, 512, 768, 1280])
def test_layernorm(dtype, D):
    L = _lib()
    rng = np.random.default_rng(D)
    rows = 333
    x = (rng.standard_normal((rows, D)) * 3 + 1).astype(np.float32)
    w = (1 + 0.1 * rng.standard_normal(D)).astype(np.float32)
    b = (0.1 * rng.standard_normal(D)).astype(np.float32)
    out = np.empty((rows, D), np.float32)
    L.check(L.lib().clipgpu_test_layernorm(dtype, rows, D, 1e-5, x.ctypes.data, w.ctypes.data, b.ctypes.data,
                                           out.ctypes.data))
    ref = clip_ref.layer_norm(x.astype(np.float64), w, b, 1e-5)
    rel = 2 ** -8 if dtype == BF16 else 2 ** -11
    assert np.all(np.abs(out - ref) <= 1.01 * rel * np.abs(ref) + 1e-5)


@pytest.mark.parametrize("mode", [0, 1])
@pytest.mark.parametrize("S,P", [(224, 32), (64, 16), (70, 14), (384, 16)])
def test_patch_rows_bit_exact(mode, S, P):
    """Staged patch rows == bf16(normalised pixels) in conv1's (ch, ky, kx) order, zero K padding;
    the u8 source normalises exactly as normalize_pixels (src/vision.rs:235-259)."""
    L = _lib()
    from oracle.model_spec import OPENAI_MEAN, OPENAI_STD
    from tests.helpers import normalized_pixels
    rng = np.random.default_rng(7 * S + mode)
    B, G, K = 2, S // P, 3 * P * P
    Kp = (K + 63) // 64 * 64
    u8 = rng.integers(0, 256, (B, S, S, 3), dtype=np.uint8)
    px = normalized_pixels(u8, OPENAI_MEAN, OPENAI_STD)
    src = px if mode == 0 else u8
    out = np.empty((B * G * G, Kp), np.float32)
    L.check(L.lib().clipgpu_test_patch_rows(BF16, mode, B, S, P, src.ctypes.data, L.f3(OPENAI_MEAN),
                                            L.f3(OPENAI_STD), out.ctypes.data))
    ref = round16(px, BF16).reshape(B, 3, G, P, G, P).transpose(0, 2, 4, 1, 3, 5).reshape(B * G * G, K)
    assert np.array_equal(out[:, :K], ref)
    assert np.all(out[:, K:] == 0)


@pytest.mark.parametrize("mode", [0, 1])
@pytest.mark.parametrize("S,P,D", [(224, 32, 768), (64, 16, 128), (70, 14, 160), (378, 14, 1280)])
def test_patch_embed(mode, S, P, D, tile):
    L = _lib()
    from oracle.model_spec import OPENAI_MEAN, OPENAI_STD
    from tests.helpers import normalized_pixels
    rng = np.random.default_rng(S + mode)
    B, G = 3, S // P
    u8 = rng.integers(0, 256, (B, S, S, 3), dtype=np.uint8)
    px = normalized_pixels(u8, OPENAI_MEAN, OPENAI_STD)
    W = round16(rng.standard_normal((D, 3 * P * P)) / np.sqrt(3 * P * P), BF16)
    pos = rng.standard_normal((G * G + 1, D)).astype(np.float32)
    out = np.empty((B * (G * G + 1), D), np.float32)
    src = px if mode == 0 else u8
    L.check(L.lib().clipgpu_test_patch_embed(BF16, mode, B, S, P, D, src.ctypes.data, L.f3(OPENAI_MEAN),
                                             L.f3(OPENAI_STD), W.ctypes.data, pos.ctypes.data, out.ctypes.data))
    pxr = round16(px, BF16).astype(np.float64)
    patches = pxr.reshape(B, 3, G, P, G, P).transpose(0, 2, 4, 1, 3, 5).reshape(B, G * G, 3 * P * P)
    ref = patches @ W.T.astype(np.float64) + pos[1:]
    got = out.reshape(B, G * G + 1, D)
    assert np.all(got[:, 0] == 0)  # CLS rows untouched
    bound = 3e-5 * (np.abs(patches) @ np.abs(W).T) + 1e-5
    assert np.all(np.abs(got[:, 1:] - ref) <= bound)


def test_lane_reductions():
    """DPP row rotations + permlane16/32 swaps (common.hpp) == the reductions they replace."""
    L = _lib()
    x = np.random.default_rng(9).standard_normal(64).astype(np.float32)
    out = np.empty(512, np.float32)
    L.check(L.lib().clipgpu_test_lane_reduce(x.ctypes.data, out.ctypes.data))
    o = out.reshape(8, 64)
    lanes = np.arange(64)
    assert np.allclose(o[0], x.sum(), rtol=1e-5)
    assert np.array_equal(o[1], np.full(64, x.max(), np.float32))
    assert np.allclose(o[2], x + x[lanes ^ 16], rtol=1e-6)
    assert np.allclose(o[3], x + x[lanes ^ 32], rtol=1e-6)
    rows = x.reshape(4, 16)
    assert np.allclose(o[4], np.repeat(rows.sum(1), 16), rtol=1e-5)
    assert np.array_equal(o[5], np.repeat(rows.max(1), 16))
    # raw permlane16 swap of (x, x): rows {0,0,2,2} and {1,1,3,3}
    assert np.array_equal(o[6], np.repeat(rows[[0, 0, 2, 2]], 1, axis=0).ravel())
    assert np.array_equal(o[7], np.repeat(rows[[1, 1, 3, 3]], 1, axis=0).ravel())
