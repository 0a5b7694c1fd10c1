"""TEST INFRASTRUCTURE ONLY: ctypes driver of the C oracle (oracle/build/libmsc_oracle.so).

Imported by tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg, always as the
CHECKER (or the timed CPU baseline), never as part of the product path. The oracle restates the
reference's env hot path (src/environment/envs/multi_env.py:192-366) in plain C; see
oracle/msc_oracle.c for the per-function reference citations.
"""
from __future__ import annotations

import ctypes as C
import subprocess
import sys
from pathlib import Path

import numpy as np

HERE = Path(__file__).resolve().parent
REPO = HERE.parent
sys.path.insert(0, str(REPO / "marl-sc_amd"))
from marlsc import abi  # noqa: E402  (descriptor struct only)
from marlsc.spec import EnvSpec  # noqa: E402

LIB_PATH = HERE / "build" / "libmsc_oracle.so"
_L = None


def build() -> None:
    subprocess.run(["make", "-s", "-C", str(HERE)], check=True)


def lib():
    global _L
    if _L is None:
        if not LIB_PATH.exists():
            build()
        L = C.CDLL(str(LIB_PATH))
        vp = C.c_void_p
        L.orc_create.argtypes = [C.POINTER(abi.MscEnvDesc), C.c_int64, C.c_uint32, C.c_uint32, C.c_int64,
                                 C.POINTER(C.c_uint32)]
        L.orc_create.restype = vp
        L.orc_destroy.argtypes = [vp]
        L.orc_error.restype = C.c_char_p
        L.orc_dims.argtypes = [vp, C.POINTER(C.c_int32), C.POINTER(C.c_int32), C.POINTER(C.c_int32)]
        L.orc_reset.argtypes = [vp, vp, vp, C.c_int32, vp]
        L.orc_step.argtypes = [vp, vp, vp, vp, vp, vp, C.POINTER(abi.MscStepInfo), C.c_int32]
        L.orc_read_state.argtypes = [vp, vp, vp, vp, vp]
        L.orc_seedseq_u32.argtypes = [C.POINTER(C.c_uint32), C.c_int32]
        L.orc_seedseq_u32.restype = C.c_uint32
        L.orc_seedseq_state.argtypes = [C.POINTER(C.c_uint32), C.c_int32, C.POINTER(C.c_uint32), C.c_int32,
                                         C.POINTER(C.c_uint32), C.c_int32]
        L.orc_rng_seed.argtypes = [vp, C.POINTER(C.c_uint32), C.c_int32, C.POINTER(C.c_uint32), C.c_int32]
        L.orc_rng_next64.argtypes = [vp]
        L.orc_rng_next64.restype = C.c_uint64
        L.orc_rng_random.argtypes = [vp]
        L.orc_rng_random.restype = C.c_double
        L.orc_rng_poisson.argtypes = [vp, C.c_double]
        L.orc_rng_poisson.restype = C.c_int64
        L.orc_rng_poisson_n.argtypes = [vp, vp, C.c_int64, C.c_int64, vp]
        L.orc_rng_poisson_n.restype = None
        L.orc_rng_integers.argtypes = [vp, C.c_int64, C.c_int64]
        L.orc_rng_integers.restype = C.c_int64
        _L = L
    return _L


def _ptr(a):
    return None if a is None else a.ctypes.data_as(C.c_void_p)


def u32s(words):
    a = (C.c_uint32 * len(words))(*[int(w) & 0xFFFFFFFF for w in words])
    return a


def seedseq_u32(words) -> int:
    return int(lib().orc_seedseq_u32(u32s(words), len(words)))


class OracleRng:
    def __init__(self, entropy, spawn_key=()):
        self.buf = (C.c_uint64 * 6)()
        ent, key = u32s(entropy), u32s(spawn_key) if spawn_key else None
        lib().orc_rng_seed(C.byref(self.buf), ent, len(entropy), key, len(spawn_key))

    @classmethod
    def from_state(cls, w):
        """A stream at a raw state [state_hi, state_lo, inc_hi, inc_lo, has32, u32]."""
        r = cls.__new__(cls)
        r.buf = (C.c_uint64 * 6)(*[int(x) for x in np.asarray(w, dtype=np.uint64)])
        return r

    def state(self):
        return np.array(list(self.buf), dtype=np.uint64)

    def poisson_n(self, lam, n: int) -> np.ndarray:
        """n draws of Generator.poisson with the rates `lam` (scalar or cycled array)."""
        lam = np.ascontiguousarray(np.atleast_1d(lam), dtype=np.float64)
        out = np.empty(int(n), dtype=np.int64)
        lib().orc_rng_poisson_n(C.byref(self.buf), _ptr(lam), lam.size, int(n), _ptr(out))
        return out

    def next64(self):
        return lib().orc_rng_next64(C.byref(self.buf))

    def random(self):
        return lib().orc_rng_random(C.byref(self.buf))

    def poisson(self, lam):
        return lib().orc_rng_poisson(C.byref(self.buf), float(lam))

    def integers(self, lo, hi):
        return lib().orc_rng_integers(C.byref(self.buf), int(lo), int(hi))


INFO_SHAPES = {
    "inventory_before": "WK", "pending_total": "WK", "order_quantities": "WK", "demand_per_region": "RK",
    "fulfilled_per_warehouse": "WK", "unfulfilled_demands": "RK", "shipment_counts": "WR",
    "shipment_quantities": "WR", "shipment_quantities_by_sku": "WRK", "lost_order_counts": "R", "n_orders": "",
    "lost_sales": "WK", "costs": "4W",
}


class OracleEnv:
    """E reference envs on the CPU with the msc_env_* semantics (auto-reset on truncation)."""

    def __init__(self, spec: EnvSpec, n_envs: int, *, base_seed: int = 0, worker_index: int = 0,
                 env_index_offset: int = 0, env_seeds=None):
        self.spec, self.E = spec, n_envs
        desc = spec.to_desc()
        seeds = None if env_seeds is None else (C.c_uint32 * n_envs)(*[int(s) for s in env_seeds])
        self.h = lib().orc_create(C.byref(desc), n_envs, base_seed, worker_index, env_index_offset, seeds)
        if not self.h:
            raise RuntimeError(lib().orc_error().decode())
        L, F, lm = C.c_int32(), C.c_int32(), C.c_int32()
        lib().orc_dims(self.h, C.byref(L), C.byref(F), C.byref(lm))
        self.L, self.F = L.value, F.value
        assert self.L == spec.local_obs_dim, (self.L, spec.local_obs_dim)

    def __del__(self):
        if getattr(self, "h", None):
            lib().orc_destroy(self.h)
            self.h = None

    def reset(self, mask=None, new_root_seeds=None, flags=0):
        obs = np.zeros((self.E, self.spec.W, self.L), np.float32)
        m = None if mask is None else np.ascontiguousarray(mask, np.uint8)
        s = None if new_root_seeds is None else np.ascontiguousarray(new_root_seeds, np.uint32)
        lib().orc_reset(self.h, _ptr(m), _ptr(s), flags, _ptr(obs))
        return obs

    def alloc_info(self):
        W, K, R = self.spec.W, self.spec.K, self.spec.R
        dims = {"W": W, "K": K, "R": R, "4": 4}
        out = {}
        for k, sh in INFO_SHAPES.items():
            shape = (self.E,) + tuple(dims[c] for c in sh)
            out[k] = np.zeros(shape, np.float64 if k in ("lost_sales", "costs") else np.int32)
        return out

    def step(self, actions, *, info=None, final_obs=False, n_threads=1):
        E, W, L = self.E, self.spec.W, self.L
        actions = np.ascontiguousarray(actions, np.float32).reshape(E, W, self.spec.K)
        obs = np.zeros((E, W, L), np.float32)
        rew = np.zeros((E, W), np.float64)
        tr = np.zeros(E, np.uint8)
        fo = np.zeros((E, W, L), np.float32) if final_obs else None
        si = None
        if info is not None:
            si = abi.MscStepInfo()
            for k, v in info.items():
                setattr(si, k, v.ctypes.data_as(C.POINTER(C.c_double if v.dtype == np.float64 else C.c_int32)))
            si = C.byref(si)
        lib().orc_step(self.h, _ptr(actions), _ptr(obs), _ptr(rew), _ptr(tr), _ptr(fo), si, n_threads)
        return obs, rew, tr.astype(bool), fo

    def read_state(self):
        E, WK = self.E, self.spec.W * self.spec.K
        inv = np.zeros((E, self.spec.W, self.spec.K), np.int32)
        ts = np.zeros(E, np.int32)
        ep = np.zeros(E, np.int32)
        rng = np.zeros((E, 2, 6), np.uint64)
        lib().orc_read_state(self.h, _ptr(inv), _ptr(ts), _ptr(ep), _ptr(rng))
        return {"inventory": inv, "timestep": ts, "episode_counter": ep, "rng": rng}
