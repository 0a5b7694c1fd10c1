"""Known-answer vectors for numpy's Poisson sampler in its PTRS branch (lam >= 10), the branch the
reference reaches whenever a config's lambda_orders / lambda_quantity is >= 10
(src/environment/components/demand_sampler.py:138,153 call Generator.poisson with any rate).

numpy only (no reference import): numpy/random/src/distributions/distributions.c, random_poisson
-> random_poisson_ptrs (Hoermann's transformed rejection, lam >= 10) / random_poisson_mult
(lam < 10), numpy 2.2.x as installed here. Each stream is Generator(PCG64(SeedSequence([7, i])))
drawn with one rate (and one stream cycling rates over both branches); the PCG64 state before and
after pins how many 64-bit words every draw consumed.
Usage: python tests/golden/make_ptrs_vectors.py  ->  tests/golden/poisson_ptrs.npz"""
from pathlib import Path

import numpy as np
from numpy.random import PCG64, Generator, SeedSequence

HERE = Path(__file__).resolve().parent
N = 100_000
RATES = [10.0, 12.5, 30.0, 100.0]
MIX = np.array([3.5, 10.0, 11.25, 0.7, 55.0, 9.999, 250.0], dtype=np.float64)


def _state(g):
    st = g.bit_generator.state
    s, inc = st["state"]["state"], st["state"]["inc"]
    return np.array([s >> 64, s & (2**64 - 1), inc >> 64, inc & (2**64 - 1), st["has_uint32"], st["uinteger"]],
                    dtype=np.uint64)


def main():
    out = {"rates": np.array(RATES), "mix_rates": MIX, "numpy_version": np.array(np.__version__)}
    for i, lam in enumerate(RATES):
        g = Generator(PCG64(SeedSequence([7, i])))
        out[f"init_{i}"] = _state(g)
        x = g.poisson(lam, size=N)
        assert x.max() < 2**15
        out[f"draws_{i}"] = x.astype(np.int16)
        out[f"final_{i}"] = _state(g)
    g = Generator(PCG64(SeedSequence([7, 99])))
    out["init_mix"] = _state(g)
    lam = np.resize(MIX, N)
    out["draws_mix"] = g.poisson(lam).astype(np.int16)
    out["final_mix"] = _state(g)
    np.savez_compressed(HERE / "poisson_ptrs.npz", **out)
    print("wrote", HERE / "poisson_ptrs.npz")


if __name__ == "__main__":
    main()
