"""Fused policy-MLP inference for the rollout (msc_mlp3_relu_forward / msc_mlp2_relu_forward,
csrc/mlp.hip).

The reference's actor / critic networks are `MLPArchitecture.build` MLPs
(src/algorithms/models/architectures/mlp.py:14-60): Linear -> ReLU per hidden size, then an output
Linear. At rollout (inference, no autograd) the ReLU MLPs of the reference's algorithm configs run
as ONE HIP kernel on the f32 MFMA with the hidden activations in registers:
* two hidden layers [H1, H2], H1, H2 in {64, 128, 256, 512} (MAPPO actor [256, 256] and critic
  [64, 64], config_files/algorithms/mappo.yaml; the test configs' [256, 256] actors);
* one hidden layer [H], H a multiple of 32 up to 1024 (IPPO actor and critic [256],
  config_files/algorithms/ippo.yaml; the test configs' [128] and [1024] critics).
The kernels stream the weights in a lane-major fragment order; `pack_mlp3` builds it from the
torch [out, in] matrices (index maps cached per shape, packs cached per weight version, so the
learner's updates are picked up and the pack is rebuilt at most once per optimizer step). A pack
built on one HIP stream and used on another is ordered by an event (rollout lanes).

There is no CPU fallback: a CUDA tensor on a build without libmarlsc raises (abi.lib()).
"""
from __future__ import annotations

import ctypes as C
import os
from typing import Dict, Optional, Tuple

import torch
import torch.nn as nn

from . import abi

HIDDEN_SIZES = (64, 128, 256, 512)  # two-hidden-layer form
MAX_HIDDEN_1 = 1024                  # one-hidden-layer form: multiples of 32 up to this
MAX_OUT = 32
MAX_IN = 1024
ENABLED = os.environ.get("MSC_FUSED_MLP3", "1") != "0"

_IDX: Dict[Tuple, Tuple[torch.Tensor, ...]] = {}


def _rho(r: torch.Tensor, h: torch.Tensor) -> torch.Tensor:
    """Row of register r in lane half h of a 32x32 f32 MFMA accumulator."""
    return (r & 3) + 8 * (r >> 2) + 4 * h


def _index_maps(L: int, H1: int, H2: int, KO: int, device, w3_layout: int) -> Tuple[torch.Tensor, ...]:
    """H2 = 0: the one-hidden-layer form (no w2; the output layer reads H1)."""
    key = (L, H1, H2, KO, str(device), w3_layout)
    if key in _IDX:
        return _IDX[key]
    KS1 = (L + 1) // 2
    M4 = (KS1 + 3) // 4
    lane = torch.arange(64, device=device)
    c, h = lane & 31, lane >> 5
    # w1p[t][m4][lane][i] = W1[32 t + c][h KS1 + m], m = 4 m4 + i  (0 for m >= KS1 or past in_dim)
    t = torch.arange(H1 // 32, device=device)[:, None, None, None]
    m = torch.arange(M4, device=device)[None, :, None, None] * 4 + torch.arange(4, device=device)[None, None, None, :]
    f = h[None, None, :, None] * KS1 + m
    i1 = ((t * 32 + c[None, None, :, None]) * L + f.clamp(max=L - 1)).reshape(-1)
    v1 = ((f < L) & (m < KS1)).expand(H1 // 32, M4, 64, 4).reshape(-1)
    # w2p[t2][s4][lane][i] = W2[32 t2 + c][32 t1 + rho(r, h)], s = 4 s4 + i = 16 t1 + r
    i2 = None
    if H2:
        S = (H1 // 32) * 16
        t2 = torch.arange(H2 // 32, device=device)[:, None, None, None]
        s = (torch.arange(S // 4, device=device)[None, :, None, None] * 4 + torch.arange(4, device=device)[None, None, None, :])
        hh = h[None, None, :, None]
        cc = c[None, None, :, None]
        i2 = ((t2 * 32 + cc) * H1 + (s // 16) * 32 + _rho(s % 16, hh)).reshape(-1)
    H2 = H2 or H1  # the output layer reads the last hidden layer
    if w3_layout == 0:
        # w3p[q][lane][i] = W3[c][32 (q // 4) + rho(4 (q % 4) + i, h)]  (0 for output rows >= KO)
        q = torch.arange((H2 // 32) * 4, device=device)[:, None, None]
        r = (q % 4) * 4 + torch.arange(4, device=device)[None, None, :]
        c3, h3 = c[None, :, None], h[None, :, None]
        i3 = (c3.clamp(max=KO - 1) * H2 + (q // 4) * 32 + _rho(r, h3)).reshape(-1)
        v3 = (c3 < KO).expand((H2 // 32) * 4, 64, 4).reshape(-1)
    else:
        # VALU output layer: w3p[s][h][a] = W3[a][32 (s // 16) + rho(s % 16, h)]  (0 for a >= KO)
        sv = torch.arange((H2 // 32) * 16, device=device)[:, None, None]
        hv = torch.arange(2, device=device)[None, :, None]
        av = torch.arange(8, device=device)[None, None, :]
        i3 = (av.clamp(max=KO - 1) * H2 + (sv // 16) * 32 + _rho(sv % 16, hv)).reshape(-1)
        v3 = (av < KO).expand((H2 // 32) * 16, 2, 8).reshape(-1)
    _IDX[key] = (i1, v1, i2, i3, v3)
    return _IDX[key]


def w3_layout(out_dim: int) -> int:
    """Packed layout of the output layer the kernel uses for out_dim outputs (msc_mlp3_w3_layout):
    0 = MFMA fragments [H2/8][64][4], 1 = VALU rows [H2/2][2][8]."""
    v = abi.lib().msc_mlp3_w3_layout(int(out_dim))
    if v < 0:
        raise ValueError(f"the fused MLP supports 1..{MAX_OUT} outputs, not {out_dim}")
    return v


def pack_mlp3(w1: torch.Tensor, w2: Optional[torch.Tensor], w3: torch.Tensor, layout: Optional[int] = None):
    """Torch Linear weights ([H1, L], [H2, H1], [KO, H2]) -> (w1p, w2p, w3p) fragment order;
    w2 None: the one-hidden-layer form ([H1, L], [KO, H1] -> (w1p, None, w3p)).
    layout: the output layer's (w3_layout(KO) when None)."""
    H1, L = w1.shape
    H2, KO = (w2.shape[0] if w2 is not None else 0), w3.shape[0]
    i1, v1, i2, i3, v3 = _index_maps(L, H1, H2, KO, w1.device, w3_layout(KO) if layout is None else layout)
    zero = torch.zeros((), device=w1.device, dtype=torch.float32)
    w1p = torch.where(v1, w1.detach().float().reshape(-1)[i1], zero)
    w2p = w2.detach().float().reshape(-1)[i2].contiguous() if w2 is not None else None
    w3p = torch.where(v3, w3.detach().float().reshape(-1)[i3], zero)
    return w1p.contiguous(), w2p, w3p.contiguous()


def fused_layers(mods) -> int:
    """2 or 3 when mods (Linear, ReLU, ..., Linear) has a fused kernel: one hidden layer of a
    multiple of 32 up to 1024 units, or two of {64, 128, 256, 512}; <= 1024 inputs, <= 32 outputs.
    0 otherwise (the caller runs the torch layers)."""
    n = len(mods)
    if n not in (3, 5):
        return 0
    lins, acts = mods[0::2], mods[1::2]
    if not all(isinstance(m, nn.Linear) and m.bias is not None for m in lins):
        return 0
    if not all(isinstance(a, nn.ReLU) for a in acts):
        return 0
    for a, b in zip(lins[:-1], lins[1:]):
        if b.in_features != a.out_features:
            return 0
    if lins[0].in_features > MAX_IN or lins[-1].out_features > MAX_OUT:
        return 0
    if n == 3:
        H = lins[0].out_features
        return 2 if (H % 32 == 0 and 32 <= H <= MAX_HIDDEN_1) else 0
    return 3 if (lins[0].out_features in HIDDEN_SIZES and lins[1].out_features in HIDDEN_SIZES) else 0


def fusable(mods) -> bool:
    return fused_layers(mods) > 0


class _Pack:
    __slots__ = ("key", "tensors", "stream", "event")

    def __init__(self):
        self.key, self.tensors, self.stream, self.event = None, None, None, None


def sample_fusable(mods) -> bool:
    """True when the fused kernel for mods can also sample the actions (VALU output layer)."""
    return fused_layers(mods) > 0 and w3_layout(mods[-1].out_features) == 1


def mlp3_forward(mods, x: torch.Tensor, out: Optional[torch.Tensor] = None, *, w1: Optional[torch.Tensor] = None,
                 pre1: Optional[torch.Tensor] = None, group: int = 1, sample=None) -> torch.Tensor:
    """The fused kernel over x [..., L] (f32 CUDA) -> [..., KO]; mods as accepted by fusable()
    (Linear-ReLU-Linear-ReLU-Linear or Linear-ReLU-Linear).
    w1: a first-layer weight to use instead of mods[0].weight (e.g. its local-feature columns);
    pre1 [rows / group, H1]: added to the first layer's pre-activation of row n as pre1[n // group].
    sample: (log_std [P, KO], logstd_floor, eps, actions, logp, clipped) -- msc_gaussian_sample fused
    into the kernel's epilogue (sample_fusable(mods) must hold); the means then go to `out` only when
    it is given (returns `out`, possibly None)."""
    nl = fused_layers(mods)
    if nl == 0:
        raise ValueError("no fused kernel for this layer sequence (see fused_layers)")
    l1, l3 = mods[0], mods[-1]
    l2 = mods[2] if nl == 3 else None
    w1 = l1.weight if w1 is None else w1
    L, KO = w1.shape[1], l3.out_features
    if x.shape[-1] != L:
        raise ValueError(f"input has {x.shape[-1]} features, the MLP expects {L}")
    # pack cache on the first Linear (one per first-layer weight view): rebuilt when any weight
    # changes (version counters) or moves
    packs = getattr(l1, "_msc_packs", None)
    if packs is None:
        packs = l1._msc_packs = {}
    pk = packs.setdefault((w1.shape, w1.stride(), w1.storage_offset()), _Pack())
    weights = (w1, l3.weight) if l2 is None else (w1, l2.weight, l3.weight)
    key = tuple((p.data_ptr(), p._version) for p in weights)
    cur = torch.cuda.current_stream(x.device)
    if pk.key != key:
        pk.tensors = pack_mlp3(w1, None if l2 is None else l2.weight, l3.weight)
        pk.key = key
        pk.stream = cur
        pk.event = torch.cuda.Event()
        pk.event.record(cur)
    elif pk.stream != cur:
        # packed on another stream (e.g. the main stream of a multi-lane rollout): order this
        # stream after the packing kernels, and keep the pack's memory alive for this stream's use
        cur.wait_event(pk.event)
        for t in pk.tensors:
            if t is not None:
                t.record_stream(cur)
    w1p, w2p, w3p = pk.tensors
    lead = x.shape[:-1]
    xf = x.reshape(-1, L)
    if xf.dtype != torch.float32 or not xf.is_contiguous():
        xf = xf.float().contiguous()
    n = xf.shape[0]
    if pre1 is not None:
        pre1 = pre1.float().contiguous()
        if group < 1 or n % group or pre1.shape != (n // group, l1.out_features):
            raise ValueError(f"pre1 must be [{n // max(group, 1)}, {l1.out_features}] for {n} rows in groups of {group}")
    vp = lambda t: None if t is None else C.c_void_p(t.data_ptr())  # noqa: E731
    st = C.c_void_p(cur.cuda_stream)
    b1, b3 = (m.bias.detach().float().contiguous() for m in (l1, l3))
    if sample is not None:
        ls, floor, eps, act, logp, clipped = sample
        for t in (ls, eps, act, logp, clipped):
            if not (t.is_cuda and t.dtype == torch.float32 and t.is_contiguous()):
                raise ValueError("sampling buffers must be contiguous float32 CUDA tensors")
        if eps.numel() != n * KO or act.numel() != n * KO or clipped.numel() != n * KO or logp.numel() != n \
                or ls.dim() != 2 or ls.shape[1] != KO:
            raise ValueError("sampling buffers do not match the MLP's rows / outputs")
        ep = abi.MscGaussianEpilogue(vp(ls), int(ls.shape[0]), C.c_float(floor), vp(eps), vp(act), vp(logp), vp(clipped))
        if l2 is None:
            abi.check(abi.lib().msc_mlp2_relu_forward_sampled(vp(xf), n, L, l1.out_features, KO, vp(w1p), vp(b1), vp(w3p),
                                                              vp(b3), vp(out), vp(pre1), int(group), C.byref(ep), st))
        else:
            b2 = l2.bias.detach().float().contiguous()
            abi.check(abi.lib().msc_mlp3_relu_forward_sampled(vp(xf), n, L, l1.out_features, l2.out_features, KO,
                                                              vp(w1p), vp(b1), vp(w2p), vp(b2), vp(w3p), vp(b3), vp(out),
                                                              vp(pre1), int(group), C.byref(ep), st))
        return None if out is None else out.reshape(*lead, KO)
    if out is None:
        out = torch.empty((n, KO), device=x.device, dtype=torch.float32)
    if l2 is None:
        abi.check(abi.lib().msc_mlp2_relu_forward(vp(xf), n, L, l1.out_features, KO, vp(w1p), vp(b1), vp(w3p), vp(b3),
                                                  vp(out), vp(pre1), int(group), st))
    else:
        b2 = l2.bias.detach().float().contiguous()
        abi.check(abi.lib().msc_mlp3_relu_forward(vp(xf), n, L, l1.out_features, l2.out_features, KO, vp(w1p), vp(b1),
                                                  vp(w2p), vp(b2), vp(w3p), vp(b3), vp(out), vp(pre1), int(group), st))
    return out.reshape(*lead, KO)
