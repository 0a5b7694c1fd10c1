"""The exactness argument of the f32-ring demand kernel (marl-sc_amd/csrc/demand_v2.hip), checked on the
host: the kernel's f32 value of each draw, its f32 Poisson chain, and the decision band around
exp(-lambda) against numpy's own f64 chain (Generator.poisson's multiplication method,
demand_sampler.py:138-156 of the reference). Outside the band the f32 chain must decide exactly as the
f64 chain does for every unit of up to 24 draws; the SKU draw (U < p) is exact on the 53-bit integer."""
import numpy as np


def kernel_f32(k53: np.ndarray) -> np.ndarray:
    """|f| of demand_v2_kernel's generator: the high word of x = k << 11 rounded to f32, the next 21 bits
    exact, one fma (emulated in f64, exact: <= 53 significant bits), rounded to f32, times 2^-53."""
    x = k53.astype(np.uint64) << np.uint64(11)
    hi = (x >> np.uint64(32)).astype(np.uint32).astype(np.float32)          # v_cvt_f32_u32 (RNE)
    lo = ((x & np.uint64(0xFFFFFFFF)).astype(np.uint32) >> np.uint32(11)).astype(np.float32)
    s = (hi.astype(np.float64) * 2.0**21 + lo.astype(np.float64)).astype(np.float32)  # fmaf
    return (s * np.float32(2.0**-53)).astype(np.float32)


def band(enlam: float, b: int = 16):
    """capi.hip: hi = f32 rounded up of exp(-lam) (1 + 2^-b), lo = f32 rounded down of exp(-lam) (1 - 2^-b)."""
    up, dn = enlam * (1 + 2.0**-b), enlam * (1 - 2.0**-b)
    hi, lo = np.float32(up), np.float32(dn)
    if float(hi) < up:
        hi = np.nextafter(hi, np.float32(np.inf))
    if float(lo) > dn:
        lo = np.nextafter(lo, np.float32(-np.inf))
    return hi, lo


def test_f32_draw_within_bound():
    rng = np.random.default_rng(0)
    k = rng.integers(0, 2**53, 2_000_000, dtype=np.int64)
    k[:64] = np.arange(64)  # tiny draws (high word zero)
    u = k.astype(np.float64) * 2.0**-53
    f = kernel_f32(k).astype(np.float64)
    nz = u > 0
    assert np.all(f[~nz] == 0)
    assert np.max(np.abs(f[nz] / u[nz] - 1)) <= 2.0**-23


def test_f32_chain_decides_as_numpy_outside_the_band():
    rng = np.random.default_rng(1)
    n, L = 400_000, 24
    k = rng.integers(0, 2**53, (n, L), dtype=np.int64)
    u = k.astype(np.float64) * 2.0**-53
    f = kernel_f32(k)
    for lam in (2.5, 4.0, 5.0, 9.5, 9.99):
        enlam = float(np.exp(-lam))
        hi, lo = band(enlam)
        P, p = np.ones(n), np.ones(n, np.float32)
        undecided = 0
        for j in range(L):
            P = P * u[:, j]                        # numpy's chain: prod *= U
            p = (p * f[:, j]).astype(np.float32)   # the kernel's f32 chain
            cont, end = p > hi, p <= lo
            assert np.all(P[cont] > enlam), (lam, j)
            assert np.all(P[end] <= enlam), (lam, j)
            undecided += int((~cont & ~end).sum())
        # the band is rare (the kernel recomputes those units exactly)
        assert undecided < 1e-4 * n * L, (lam, undecided)


def test_sku_draw_exact_on_the_integer():
    # U = k 2^-53 < p  <=>  k < ceil(p 2^53)  (capi.hip v2_k53), for probabilities near representable edges
    rng = np.random.default_rng(2)
    for p in (0.3, 0.667, 0.5, 1.0, 1e-9, np.nextafter(0.5, 1), np.nextafter(0.5, 0)):
        k53 = int(np.ceil(np.ldexp(p, 53)))
        m = int(np.floor(np.ldexp(p, 53)))
        ks = np.unique(np.clip(np.concatenate([rng.integers(0, 2**53, 1000), np.arange(m - 3, m + 4)]), 0, 2**53 - 1))
        u = ks.astype(np.float64) * 2.0**-53
        assert np.array_equal(u < p, ks < k53), p
