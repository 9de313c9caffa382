"""Exact rewrites in the kernels, checked bit for bit on the CPU.

1. The tail of hash() (raytracer.glsl:302-306) as rt0_integrator.h evaluates
it: u2f(m) * 2^-32, where u2f converts m >= 2^31 the way the reference
executor does (float(m - 2^31) + 2^31, two roundings), is computed as
fma(float(m mod 2^31), 2^-32, 0.5 if m >= 2^31 else 0).  The product is exact,
so the fma's single rounding equals u2f's addition scaled by 2^-32.  Checked
here bit for bit on every boundary and 2^24 random words (an exhaustive
C sweep over all 2^32 words gave 0 mismatches).  On the GPU the per-pixel
fixture tests pin the kernel's stream (tests/test_gpu_parity.py: one wrong
hash bit decorrelates every path)."""
import numpy as np


def u2f_scaled(m):
    """The reference form: u2f(m) * 2^-32 in float32 steps."""
    lo = (m & 0x7FFFFFFF).astype(np.int32).astype(np.float32)
    hi = np.where(m >= 0x80000000, np.float32(2147483648.0), np.float32(0.0)).astype(np.float32)
    u = np.where(m >= 0x80000000, (lo + hi).astype(np.float32), m.astype(np.int64).astype(np.float32))
    return (u * np.float32(2.3283064365386963e-10)).astype(np.float32)


def fma_form(m):
    """rt0_integrator.h hash(): fma(float(m & 0x7fffffff), 2^-32, hi) with one rounding."""
    lo = (m & 0x7FFFFFFF).astype(np.int32).astype(np.float32)
    hi = np.where(m >= 0x80000000, 0.5, 0.0)
    exact = lo.astype(np.float64) * 2.0 ** -32 + hi  # exact in float64 (<= 33 significant bits)
    return exact.astype(np.float32)


def test_hash_tail_fma_is_bit_identical():
    rng = np.random.default_rng(7)
    edges = np.array([0, 1, 2, 0x7FFFFF, 0x1000000, 0x1000001, 0x7FFFFFBF, 0x7FFFFFC0, 0x7FFFFFFF, 0x80000000,
                      0x80000001, 0x80000040, 0x80000080, 0xFFFFFF7F, 0xFFFFFF80, 0xFFFFFFFF], dtype=np.uint64)
    m = np.concatenate([edges, rng.integers(0, 2 ** 32, size=1 << 24, dtype=np.uint64)])
    a, b = u2f_scaled(m), fma_form(m)
    assert (a.view(np.uint32) == b.view(np.uint32)).all()


def test_quot_small_matches_integer_division():
    """2. rt0_integrator.h quot_small: floor(a / d) as (int)((a + 0.5f) * fl(1/d))
    in float32 (row_local's band and owner of a reservoir row, sharded
    ReSTIR), exact for 0 <= a < 2^21 (a C sweep of every d <= 8192 gave 0
    mismatches); here every d <= 512 against a grid of a."""
    a = np.concatenate([np.arange(0, 1 << 14), np.arange(1 << 14, 1 << 21, 97), [(1 << 21) - 1]]).astype(np.int64)
    af = (a.astype(np.float32) + np.float32(0.5)).astype(np.float32)
    for d in range(1, 513):
        inv = np.float32(1.0) / np.float32(d)
        q = (af * inv).astype(np.float32).astype(np.int64)
        assert (q == a // d).all(), d
