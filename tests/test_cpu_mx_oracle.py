"""oracle/mx_ref.py (the MX-fp8 restatement the GPU fp8 path is checked against), on the CPU.

Pins: the e4m3 encoder round-trips every code and matches the gfx950 conversion results
recorded by tools/mx_probe.hip (RNE at midpoints, saturation to 448 = 0x7E, signed zero);
the block exponent is the smallest e with amax <= 448 * 2^e; quantize -> dequantize error is
at most half an e4m3 step at the block's top binade.
"""
import numpy as np

from oracle import mx_ref


def test_e4m3_roundtrip_every_code():
    t = mx_ref.e4m3_decode_table()
    ok = ~np.isnan(t)
    codes = np.arange(256, dtype=np.uint8)[ok]
    np.testing.assert_array_equal(mx_ref.e4m3_encode(t[ok].astype(np.float32)), codes)
    assert t[0x7E] == 448.0 and t[0x01] == 2.0 ** -9 and np.isnan(t[0x7F]) and np.isnan(t[0xFF])


def test_e4m3_known_conversions():
    # values and codes from the gfx950 v_cvt_pk_fp8_f32 probe (tools/mx_probe.hip)
    x = np.array([461.44, -461.44, -0.0009765625, 2.0 ** -10, 3 * 2.0 ** -11, 1.9375, 0.0], np.float32)
    np.testing.assert_array_equal(mx_ref.e4m3_encode(x), [0x7E, 0xFE, 0x80, 0x00, 0x01, 0x40, 0x00])


def test_midpoints_round_to_even():
    t = mx_ref.e4m3_decode_table()
    for c in range(0, 0x7D):
        mid = np.float32(0.5 * (t[c] + t[c + 1]))
        got = int(mx_ref.e4m3_encode(np.array([mid]))[0])
        assert got == (c if c % 2 == 0 else c + 1), (c, mid, got)


def test_block_exponent_rule():
    rng = np.random.default_rng(0)
    amax = np.abs(rng.standard_normal(10000)).astype(np.float32) * np.exp2(rng.integers(-30, 30, 10000)).astype(np.float32)
    e = mx_ref.mx_exp(amax)
    assert np.all(amax.astype(np.float64) <= 448.0 * np.exp2(e.astype(np.float64)))
    assert np.all(amax.astype(np.float64) > 448.0 * np.exp2(e.astype(np.float64) - 1))
    # exact boundaries
    np.testing.assert_array_equal(mx_ref.mx_exp(np.array([448.0, 448.00003, 224.0, 0.0], np.float32)), [0, 1, -1, -127])


def test_quantize_dequantize_error_bound():
    rng = np.random.default_rng(1)
    x = (rng.standard_normal((64, 256)) * np.exp2(rng.integers(-8, 8, (64, 1)))).astype(np.float32)
    q, s = mx_ref.quantize_rows(x)
    d = mx_ref.dequantize(q, s)
    half = np.ldexp(1.0, s.astype(np.int64) - 127 + 4).repeat(32, -1)
    assert np.all(np.abs(d - x) <= half)
    assert np.all(np.abs(mx_ref.e4m3_decode_table()[q]) <= 448.0)
