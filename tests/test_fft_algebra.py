"""CPU restatement of the register-form FFT decompositions the packed front half uses (rsl_fft.hip), checked against
numpy's 2-D FFT: the index algebra of each kernel pair, not its rounding (that is the GPU parity tests' job).
  S = 512,  C = 128: k_range_fft_r512 (16 x 32: DFT16 over m, DFT16 over j = 2 i + h, radix-2 across the lane pair),
                     Doppler step W128^(c k1) DFT8 over q (chirps c + 16 q), k_doppler_detect_r128 DFT16 over classes;
  S = 1024, C = 256: k_range_fft_r1024 (16 x 64: DFT16 over m, DFT16 over j = 4 i + h, radix-4 across the lane quad
                     as two swaps (h ^ 2, then h ^ 1 after the W4 twiddle), lane h ending with s = (h >> 1) | 2 (h & 1)),
                     W256^(c k1) DFT8 over q (chirps c + 32 q), k_doppler_detect_r256 DFT32 over classes as DFT16 over
                     c = 2 i + h and a radix-2 step;
  S = 256,  C = 64:  k_range_fft_r256 (16 x 16, no cross-lane step), W64^(c k1) DFT8 over q (chirps c + 8 q),
                     k_doppler_detect_r64 DFT8 over classes."""
import numpy as np
import pytest

W = lambda n, N: np.exp(-2j * np.pi * np.asarray(n) / N)


def range_r512(x):
    V = np.array([np.fft.fft(x[j::32]) * W(j * np.arange(16), 512) for j in range(32)])  # V[j][k1]
    X = np.zeros(512, complex)
    for k1 in range(16):
        E = np.fft.fft(V[0::2, k1])  # lane h = 0: j = 2 i
        O = np.fft.fft(V[1::2, k1])  # lane h = 1: j = 2 i + 1
        Wk = W(np.arange(16), 32)
        X[k1 + 16 * np.arange(16)] = E + Wk * O
        X[k1 + 16 * (np.arange(16) + 16)] = E - Wk * O
    return X


def range_r1024(x):
    V = np.array([np.fft.fft(x[j::64]) * W(j * np.arange(16), 1024) for j in range(64)])  # V[j][k1]
    X = np.zeros(1024, complex)
    for k1 in range(16):
        F = [np.fft.fft(V[h::4, k1]) for h in range(4)]  # lane h: DFT16 over j = 4 i + h
        u = [F[h] * W(h * np.arange(16), 64) for h in range(4)]  # W64^(h k)
        a = [None] * 4
        for h in range(4):  # swap with h ^ 2: lanes with h & 2 hold the difference
            a[h] = u[h] + u[h ^ 2] if not h & 2 else u[h ^ 2] - u[h]
        for h in (3,):  # W4^(s0) = -i on the lane with h0 = 1, s0 = 1
            a[h] = -1j * a[h]
        for h in range(4):  # swap with h ^ 1
            y = a[h] + a[h ^ 1] if not h & 1 else a[h ^ 1] - a[h]
            s = (h >> 1) | ((h & 1) << 1)
            X[k1 + 16 * np.arange(16) + 256 * s] = y
    return X


def range_r256(x):
    V = np.array([np.fft.fft(x[j::16]) * W(j * np.arange(16), 256) for j in range(16)])
    X = np.zeros(256, complex)
    for k1 in range(16):
        X[k1 + 16 * np.arange(16)] = np.fft.fft(V[:, k1])
    return X


def doppler(Xr, ncls, rows):
    """K1's Doppler step per class c (chirps c + ncls q, q < rows): Y_c[k1] = W_C^(c k1) DFT_rows over q; then K2's
    DFT over the classes: X[k1 + rows k2] = DFT_ncls over c of Y_c[k1]."""
    C = ncls * rows
    Y = np.array([np.fft.fft(Xr[c::ncls], axis=0) * W(c * np.arange(rows), C)[:, None] for c in range(ncls)])
    out = np.zeros_like(Xr)
    for k1 in range(rows):
        if ncls == 32:  # k_doppler_detect_r256: DFT16 over c = 2 i + h, radix-2 across the lane pair
            E, O = np.fft.fft(Y[0::2, k1], axis=0), np.fft.fft(Y[1::2, k1], axis=0)
            Wk = W(np.arange(16), 32)[:, None]
            out[k1 + rows * np.arange(16)] = E + Wk * O
            out[k1 + rows * (np.arange(16) + 16)] = E - Wk * O
        else:
            out[k1 + rows * np.arange(ncls)] = np.fft.fft(Y[:, k1], axis=0)
    return out


@pytest.mark.parametrize('shape', [(128, 512), (256, 1024), (64, 256)])
def test_register_form_decomposition(shape):
    C, S = shape
    rs = np.random.RandomState(C)
    x = rs.randn(C, S) + 1j * rs.randn(C, S)
    rf = {512: range_r512, 1024: range_r1024, 256: range_r256}[S]
    Xr = np.array([rf(row) for row in x])
    np.testing.assert_allclose(Xr, np.fft.fft(x, axis=1), atol=1e-9 * np.abs(Xr).max())
    ncls = {128: 16, 256: 32, 64: 8}[C]
    got = doppler(Xr, ncls, 8)
    np.testing.assert_allclose(got, np.fft.fft2(x), atol=1e-9 * np.abs(got).max())
