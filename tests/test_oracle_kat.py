"""Known-answer tests pinning every TF semantic the CPU restatement could get wrong (SURVEY.md
Appendix A). Hand-derived values — the reference itself cannot run here (TensorFlow absent) and ships no
tests or fixtures, so these are what pins the oracle."""
import math

import numpy as np
import pytest
import torch

from oracle import reset_perm
from oracle import vqvae_ref as R


def t(a):
    return torch.tensor(a, dtype=torch.float64)


@pytest.mark.parametrize("T,K,s,d,want", [(4096, 4, 2, 1, (2048, 1, 1)), (4097, 4, 2, 1, (2049, 1, 2)),
                                          (512, 3, 1, 27, (512, 27, 27)), (40, 3, 1, 27, (40, 27, 27)),
                                          (7, 3, 1, 1, (7, 1, 1)), (65536, 4, 2, 1, (32768, 1, 1))])
def test_same_padding(T, K, s, d, want):
    """A.2: out = ceil(T/s); pad = max((out-1)s + (K-1)d + 1 - T, 0); left = pad // 2."""
    assert R.same_pad(T, K, s, d) == want


def test_conv1d_same_known_answer():
    x = t([1, 2, 3, 4]).reshape(1, 4, 1)
    W = t([1, 10, 100]).reshape(3, 1, 1)
    y = R.conv1d(x, W, t([0.0]), 1, 1)
    assert y.reshape(-1).tolist() == [210, 321, 432, 43]  # x[t-1] + 10 x[t] + 100 x[t+1]


def test_conv1d_dilated_known_answer():
    x = t(np.arange(1, 9)).reshape(1, 8, 1)
    W = t([1, 10, 100]).reshape(3, 1, 1)
    y = R.conv1d(x, W, t([0.5]), 1, 3)  # pad (3, 3): x[t-3] + 10 x[t] + 100 x[t+3] + 0.5
    assert y.reshape(-1).tolist() == [410.5, 520.5, 630.5, 741.5, 852.5, 63.5, 74.5, 85.5]


def test_conv1d_strided_known_answer():
    x = t(np.arange(1, 9)).reshape(1, 8, 1)
    W = t([1, 10, 100, 1000]).reshape(4, 1, 1)
    y = R.conv1d(x, W, t([0.0]), 2, 1)  # pad (1, 1): y[t] = sum_k x[2t + k - 1] W[k]
    assert y.reshape(-1).tolist() == [3210, 5432, 7654, 876]


def test_conv1d_channels_layout():
    """Keras kernel (K, C_in, C_out): y[t, o] = sum_{k,c} x[t+k-1, c] W[k, c, o]."""
    rng = np.random.default_rng(0)
    x, W = rng.standard_normal((1, 5, 2)), rng.standard_normal((3, 2, 3))
    y = R.conv1d(t(x), t(W), t(np.zeros(3)), 1, 1).numpy()
    xp = np.pad(x[0], ((1, 1), (0, 0)))
    want = np.stack([sum(xp[i + k] @ W[k] for k in range(3)) for i in range(5)])
    assert np.allclose(y[0], want)


def test_conv1d_transpose_alignment():
    """A.3: Conv1DTranspose(K=4, s=2, same) is the adjoint of the SAME conv: pad_left 1, length 2T."""
    x = t([0, 1, 0, 0]).reshape(1, 4, 1)
    W = t([1, 10, 100, 1000]).reshape(4, 1, 1)
    y = R.conv1d_transpose(x, W, t([0.0]), 2)
    assert y.reshape(-1).tolist() == [0, 1, 10, 100, 1000, 0, 0, 0]
    # adjoint identity <convT(x), y> == <x, conv(y)> with the same kernel (layouts (K,Cout,Cin) vs (K,Cin,Cout))
    rng = np.random.default_rng(1)
    xx, yy, WW = rng.standard_normal((2, 6, 3)), rng.standard_normal((2, 12, 5)), rng.standard_normal((4, 5, 3))
    lhs = (R.conv1d_transpose(t(xx), t(WW), t(np.zeros(5)), 2) * t(yy)).sum()
    rhs = (t(xx) * R.conv1d(t(yy), t(WW), t(np.zeros(3)), 2, 1)).sum()
    assert abs(float(lhs - rhs)) < 1e-9


@pytest.mark.parametrize("T,want", [(4096, (13, 30, 78)), (65536, (269, 542, 1306)), (2048, (4, 13, 37))])
def test_stft_frame_counts(T, want):
    """A.4: frames = 1 + (T - win) // hop, no centering, pad_end=False."""
    x = torch.zeros(T, dtype=torch.float64)
    got = tuple(R.spectral(x, n_fft, hop, win).shape[0] for n_fft, hop, win in R.STFT_ARGS)
    assert got == want
    assert tuple(R.spectral(x, n_fft, hop, win).shape[1] for n_fft, hop, win in R.STFT_ARGS) == (1025, 513, 257)


def test_hann_periodic():
    assert np.allclose(R.hann_periodic(4).numpy(), [0, 0.5, 1, 0.5])


def test_stft_framing_and_zero_padding():
    """frame t starts at t*hop; the windowed frame is zero-padded at the END to n_fft."""
    T, win, hop, n_fft = 64, 8, 4, 16
    x = torch.arange(T, dtype=torch.float64)
    S = R.spectral(x, n_fft, hop, win)
    w = R.hann_periodic(win).numpy()
    f3 = np.zeros(n_fft)
    f3[:win] = np.arange(12, 20) * w
    assert np.allclose(S[3].numpy(), np.abs(np.fft.rfft(f3)))
    # a constant signal: DC bin = sum of the window = win / 2
    S1 = R.spectral(torch.ones(T, dtype=torch.float64), n_fft, hop, win)
    assert np.allclose(S1[:, 0].numpy(), win / 2)


def test_multispectral_loss_definition():
    rng = np.random.default_rng(2)
    x, r = t(rng.standard_normal((2, 4096, 1))), t(rng.standard_normal((2, 4096, 1)))
    got = R.multispectral_loss(x, r).numpy()
    want = []
    for b in range(2):
        ls = []
        for n_fft, hop, win in R.STFT_ARGS:
            sx, sr = R.spectral(x[b, :, 0], n_fft, hop, win), R.spectral(r[b, :, 0], n_fft, hop, win)
            ls.append(float(torch.linalg.norm(sx - sr) / torch.linalg.norm(sx)))
        want.append(np.mean(ls))
    assert np.allclose(got, want)
    assert float(R.multispectral_loss(x, x).sum()) == 0.0


def test_argmin_ties_lowest_index():
    """A.5: tf.argmin -> int64, first minimal index."""
    d = torch.tensor([[3.0, 1.0, 1.0, 2.0], [5.0, 5.0, 5.0, 5.0]])
    assert torch.argmin(d, dim=1).tolist() == [1, 0]


def test_keras_adam_single_step():
    """A.8: alpha = lr sqrt(1-b2^t)/(1-b1^t); eps after the bias correction."""
    w, m, v = R.keras_adam(t([1.0]), t([1.0]), t([0.0]), t([0.0]), 1)
    alpha = 1e-3 * math.sqrt(1 - 0.999) / (1 - 0.9)
    want = 1.0 - alpha * 0.1 / (math.sqrt(0.001) + 1e-7)
    assert abs(float(w) - want) < 1e-15 and abs(float(m) - 0.1) < 1e-15 and abs(float(v) - 0.001) < 1e-15
    # differs from PyTorch's Adam (eps added to sqrt(v_hat)) — that is the point of restating it
    torch_like = 1.0 - 1e-3 * 1.0 / (1.0 + 1e-8)
    assert abs(want - torch_like) > 1e-9


def test_ema_constants_float32():
    """TF multiplies float32 by the python floats gamma and (1. - gamma) -> float32(0.99), float32(0.01...)."""
    cfg = R.RefConfig(input_len=2048, levels=1, latent_dim=4, down_depth=[1], strides=[2], num_embeddings=8,
                      residual_width=8, residual_depth=1)
    m = R.RefVQVAE(cfg, R.init_params(cfg), R.init_vq_state(cfg), dtype=torch.float32)
    assert m.gamma == float(np.float32(0.99)) and m.omg == float(np.float32(1.0 - 0.99))


def _tiny_vq_model(K=8, D=2):
    cfg = R.RefConfig(input_len=2048, levels=1, latent_dim=D, down_depth=[1], strides=[2], num_embeddings=K,
                      residual_width=8, residual_depth=1)
    return R.RefVQVAE(cfg, R.init_params(cfg), R.init_vq_state(cfg), dtype=torch.float64)


def test_straight_through_value_is_z_plus_difference():
    """A.6: decoder input = z + sg(q - z) computed in the working precision, not q."""
    m = _tiny_vq_model()
    m.dtype = torch.float32
    E = torch.zeros(2, 8, dtype=torch.float32)
    E[:, 3] = torch.tensor([0.1, 0.1])
    m.vq[0]["embeddings"] = E
    z = torch.tensor([[[1024.0, 0.0]]], dtype=torch.float32)
    q_st, idx, _ = m.vq_forward(z, 0, training=False)
    q = E.T[idx]
    assert torch.equal(q_st.reshape(1, 2), z.reshape(1, 2) + (q - z.reshape(1, 2)))
    assert int(idx) == 3
    assert float(q_st.reshape(-1)[0]) != float(q.reshape(-1)[0])  # 1024 + (0.1 - 1024) != 0.1 in fp32


def test_ema_update_and_dead_code_reset():
    """VectorQuantizer.py:116-145: EMA of sums/counts; codes with N_t < 1 take reset rows; their m_t/N_t
    are NOT reset. With N_t starting at ones, every code unused in the first batch is dead after it."""
    m = _tiny_vq_model(K=8, D=2)
    E0 = m.vq[0]["embeddings"].clone()
    z = torch.tensor([[[0.04, 0.04], [0.05, 0.05], [-0.04, -0.04], [0.3, 0.3], [0.02, -0.02]]], dtype=torch.float64)
    q_st, idx, info = m.vq_forward(z, 0, training=True)
    st = m.vq[0]
    n_sum = torch.bincount(idx, minlength=8).double()
    assert torch.allclose(info["n_sum"], n_sum)
    assert torch.allclose(st["N_t"], 0.99 + 0.01 * n_sum)
    flat = z.reshape(-1, 2)
    m_sum = torch.zeros(2, 8, dtype=torch.float64)
    for i, k in enumerate(idx.tolist()):
        m_sum[:, k] += flat[i]
    assert torch.allclose(st["m_t"], 0.99 * E0 + 0.01 * m_sum)
    rows = reset_perm.reset_rows(3, 0, 0, 5, 8)  # N=5 < K=8: tiled batch
    for k in range(8):
        if n_sum[k] >= 1:
            assert torch.allclose(st["embeddings"][:, k], st["m_t"][:, k] / st["N_t"][k])
        else:
            assert torch.equal(st["embeddings"][:, k], flat[rows[k]])
    assert info["batch_usage"] == float((n_sum >= 1).sum()) and info["usage"] == info["batch_usage"]


def test_glorot_uniform_limits():
    cfg = R.RefConfig(input_len=65536, levels=3, latent_dim=64, down_depth=[3, 2, 2], strides=[2, 2, 2],
                      num_embeddings=2048, residual_width=32, residual_depth=4, dilation_factor=3)
    p = R.init_params(cfg, 1)
    for name, arr in p.items():
        if name.endswith("kernel"):
            K, a, b = arr.shape
            assert np.abs(arr).max() <= math.sqrt(6.0 / (K * a + K * b)) + 1e-7
        else:
            assert not arr.any()
    assert sum(a.size for a in p.values()) == 968835 and len(p) == 570
