"""Host test of the fused policy MLP's weight packing (marlsc/mlp.py:pack_mlp3): a numpy emulation of
the kernel's v_mfma_f32_32x32x2_f32 data flow (csrc/mlp.hip) over the packed fragments reproduces
the torch MLP (float64), so the lane / register maps of the packing are checked without a GPU.
MFMA operand maps (cdna_hip_programming.md, f32 32x32x2): lane l holds A[l & 31][k = l >> 5] and
B[k = l >> 5][l & 31]; accumulator register r of lane l is D[(r & 3) + 8 (r >> 2) + 4 (l >> 5)][l & 31]."""
import numpy as np
import pytest
import torch

from marlsc.mlp import fusable, pack_mlp3
from marlsc.rollout import MLP


def _mfma(a_lane, b_lane, d):
    A = np.zeros((32, 2))
    B = np.zeros((2, 32))
    for lane in range(64):
        A[lane & 31, lane >> 5] = a_lane[lane]
        B[lane >> 5, lane & 31] = b_lane[lane]
    return d + A @ B


def _rho(r, h):
    return (r & 3) + 8 * (r >> 2) + 4 * h


def _regs(tile, r):
    """Register r of every lane of a [32 rows x 32 samples] accumulator tile."""
    return np.array([tile[_rho(r, lane >> 5), lane & 31] for lane in range(64)])


def _emulate(mlp, x, layout=0):
    l1, _, l2, _, l3 = list(mlp)
    H1, L = l1.weight.shape
    H2, KO = l2.weight.shape[0], l3.weight.shape[0]
    KS1 = (L + 1) // 2
    M4 = (KS1 + 3) // 4
    w1p, w2p, w3p = (t.double().numpy() for t in pack_mlp3(l1.weight, l2.weight, l3.weight, layout))
    w1p = w1p.reshape(H1 // 32, M4, 64, 4)
    w2p = w2p.reshape(H2 // 32, H1 // 8, 64, 4)
    b1, b2, b3 = (m.bias.detach().double().numpy() for m in (l1, l2, l3))
    n = x.shape[0]
    assert n == 32  # one wave
    h1 = []
    for t in range(H1 // 32):
        d = np.zeros((32, 32))
        for m in range(M4 * 4):
            xb = [x[lane & 31, (lane >> 5) * KS1 + m] if m < KS1 and (lane >> 5) * KS1 + m < L else 0.0
                  for lane in range(64)]
            d = _mfma(w1p[t, m // 4, :, m % 4], xb, d)
        h1.append(np.maximum(d + b1[t * 32:(t + 1) * 32, None], 0))
    h2 = []
    for t2 in range(H2 // 32):
        d = np.zeros((32, 32))
        for s in range((H1 // 32) * 16):
            d = _mfma(w2p[t2, s // 4, :, s % 4], _regs(h1[s // 16], s % 16), d)
        h2.append(np.maximum(d + b2[t2 * 32:(t2 + 1) * 32, None], 0))
    if layout == 1:  # VALU output layer: lane half h sums its rows rho(r, h) of every tile
        w3v = w3p.reshape((H2 // 32) * 16, 2, 8)
        o = np.zeros((64, 8))
        for s in range((H2 // 32) * 16):
            hv = _regs(h2[s // 16], s % 16)
            for lane in range(64):
                o[lane] += w3v[s, lane >> 5] * hv[lane]
        return o[:32, :KO] + o[32:, :KO] + b3[None, :]
    w3p = w3p.reshape(H2 // 8, 64, 4)
    d = np.zeros((32, 32))
    for q in range((H2 // 32) * 4):
        for i in range(4):
            d = _mfma(w3p[q, :, i], _regs(h2[q // 4], (q % 4) * 4 + i), d)
    return (d[:KO] + b3[:, None]).T


@pytest.mark.parametrize("layout", [0, 1])
@pytest.mark.parametrize("L,H,KO", [(34, 64, 5), (7, 64, 1), (42, 128, 3)])
def test_packed_fragments_reproduce_the_mlp(L, H, KO, layout):
    torch.manual_seed(L * H + KO)
    mlp = MLP(L, KO, {"hidden_sizes": [H, H]})
    assert fusable(list(mlp))
    x = torch.randn(32, L, dtype=torch.float64)
    got = _emulate(mlp, x.numpy(), layout)
    ref = mlp.double()(x).detach().numpy()
    np.testing.assert_allclose(got, ref, rtol=1e-12, atol=1e-12)


def test_fusable_shapes():
    from marlsc.mlp import fused_layers
    assert fused_layers(list(MLP(34, 5, {"hidden_sizes": [256, 256]}))) == 3
    assert fused_layers(list(MLP(34, 5, {"hidden_sizes": [256, 128]}))) == 3   # unequal two-layer sizes
    assert fused_layers(list(MLP(34, 5, {"hidden_sizes": [512, 64]}))) == 3
    assert fused_layers(list(MLP(34, 5, {"hidden_sizes": [256]}))) == 2        # the reference IPPO nets
    assert fused_layers(list(MLP(306, 1, {"hidden_sizes": [1024]}))) == 2      # mappo_test critic
    assert not fusable(list(MLP(34, 5, {"hidden_sizes": [96, 96]})))      # two-layer: 64 / 128 / 256 / 512
    assert not fusable(list(MLP(34, 5, {"hidden_sizes": [1056]})))        # one layer: <= 1024
    assert not fusable(list(MLP(34, 5, {"hidden_sizes": [100]})))         # one layer: multiples of 32
    assert not fusable(list(MLP(34, 40, {"hidden_sizes": [64, 64]})))     # > 32 outputs
    assert not fusable(list(MLP(34, 5, {"hidden_sizes": [64, 64], "activation": "tanh"})))
    assert not fusable(list(MLP(1100, 5, {"hidden_sizes": [64, 64]})))    # > 1024 inputs


def test_mlp3_abi_rejects_bad_arguments_before_any_launch():
    # msc_mlp3_relu_forward validates its arguments on the host (no HIP call is made on these paths)
    import ctypes as C
    from marlsc import abi
    L = abi.lib()
    f = L.msc_mlp3_relu_forward
    p = C.c_void_p(16)  # never dereferenced: every call below fails validation first
    assert f(None, 8, 34, 256, 256, 5, p, p, p, p, p, p, p, None, 1, None) == -1
    assert b"null" in L.msc_last_error()
    assert f(p, 8, 34, 256, 96, 5, p, p, p, p, p, p, p, None, 1, None) == -1
    assert b"hidden sizes" in L.msc_last_error()
    assert f(p, 8, 34, 96, 96, 5, p, p, p, p, p, p, p, None, 1, None) == -1
    assert f(p, 8, 34, 64, 64, 33, p, p, p, p, p, p, p, None, 1, None) == -1
    assert b"out_dim" in L.msc_last_error()
    assert f(p, 8, 34, 64, 64, 5, p, p, p, p, p, p, p, p, 0, None) == -1
    assert b"pre1_group" in L.msc_last_error()
    q = C.c_void_p(20)  # misaligned bias
    assert f(p, 8, 34, 64, 64, 5, p, q, p, p, p, p, p, None, 1, None) == -1
    assert b"aligned" in L.msc_last_error()
    g = L.msc_mlp2_relu_forward  # the one-hidden-layer form
    assert g(None, 8, 34, 256, 5, p, p, p, p, p, None, 1, None) == -1
    assert b"null" in L.msc_last_error()
    assert g(p, 8, 34, 100, 5, p, p, p, p, p, None, 1, None) == -1
    assert b"hidden size" in L.msc_last_error()
    assert g(p, 8, 34, 2048, 5, p, p, p, p, p, None, 1, None) == -1
    assert g(p, 8, 2000, 256, 5, p, p, p, p, p, None, 1, None) == -1
    assert b"in_dim" in L.msc_last_error()


def test_sampled_mlp_entry_points_validate_arguments():
    # msc_mlp{3,2}_relu_forward_sampled reject a missing epilogue, missing sampling buffers and
    # output layers the epilogue does not cover (> 8 outputs) before any launch
    import ctypes as C
    from marlsc import abi
    L = abi.lib()
    p = C.c_void_p(256)
    ep = abi.MscGaussianEpilogue(p, 1, C.c_float(-3.5), p, p, p, p)
    f = L.msc_mlp3_relu_forward_sampled
    assert f(p, 8, 34, 256, 256, 5, p, p, p, p, p, p, None, None, 1, None, None) == -1
    assert b"null" in L.msc_last_error()
    assert f(p, 8, 34, 256, 256, 9, p, p, p, p, p, p, None, None, 1, C.byref(ep), None) == -1
    assert b"VALU output layer" in L.msc_last_error()
    bad = abi.MscGaussianEpilogue(p, 0, C.c_float(-3.5), p, p, p, p)
    assert f(p, 8, 34, 256, 256, 5, p, p, p, p, p, p, None, None, 1, C.byref(bad), None) == -1
    assert b"log_std_rows" in L.msc_last_error()
    g = L.msc_mlp2_relu_forward_sampled
    nul = abi.MscGaussianEpilogue(p, 1, C.c_float(-3.5), None, p, p, p)
    assert g(p, 8, 34, 256, 5, p, p, p, p, None, None, 1, C.byref(nul), None) == -1
    assert b"null sampling buffer" in L.msc_last_error()
    assert L.msc_mlp3_relu_forward(p, 8, 34, 256, 256, 5, p, p, p, p, p, p, None, None, 1, None) == -1  # out required


def test_output_layer_layout_rule():
    from marlsc.mlp import w3_layout
    assert [w3_layout(k) for k in (1, 5, 8)] == [1, 1, 1]  # VALU output layer up to 8 outputs
    assert [w3_layout(k) for k in (9, 32)] == [0, 0]       # MFMA tile beyond
    with pytest.raises(ValueError):
        w3_layout(33)
