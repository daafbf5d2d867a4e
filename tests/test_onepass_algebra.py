"""CPU check of the one-pass 64k decomposition that fft_1p_kernel (sdrpp_amd/csrc/fft.hip) runs:
a radix-4 decimation-in-frequency step X[4 m + r] = DFT_16384(y_r)[m], then each 16k transform as
radix 32 over i (n = t + 512 i) with the twiddle W_N^(t (4 k2 + r)), radix 32 over t1 (t = t0 + 16 t1)
with W_512^(t0 q1), radix 16 over t0, output m = k2 + 32 q1 + 1024 q2 -- the same index algebra as
the kernel's three stages, in fp64 numpy, against numpy's FFT of the whole frame."""
import numpy as np


def W(m, L):
    return np.exp(-2j * np.pi * (np.asarray(m) % L) / L)


def onepass_bins(x, r):
    N, M = 65536, 16384
    t = np.arange(512)[:, None]
    i = np.arange(32)[None, :]
    u = [x[t + 512 * i + M * j] for j in range(4)]
    s = (-1) ** r
    z = (u[0] + s * u[2]) + W(r, 4) * (u[1] + s * u[3])       # sum_j W_4^(j r) u_j
    z = z * W(512 * r * i, N)                                  # W_128^(r i)
    k2 = np.arange(32)[None, :]
    A = np.fft.fft(z, axis=1) * W(t * (4 * k2 + r), N)         # stage 1: [t][k2]
    A = A.reshape(32, 16, 32)                                  # [t1][t0][k2]
    q1 = np.arange(32)[:, None, None]
    t0 = np.arange(16)[None, :, None]
    B = np.fft.fft(A, axis=0) * W(128 * t0 * q1, N)            # stage 2: [q1][t0][k2]
    C = np.fft.fft(B, axis=1)                                  # stage 3: [q1][q2][k2]
    q2 = np.arange(16)[None, :, None]
    m = np.arange(32)[None, None, :] + 32 * q1 + 1024 * q2
    Y = np.empty(M, complex)
    Y[m.ravel()] = C.ravel()
    return Y


def test_onepass_index_algebra():
    rng = np.random.default_rng(3)
    x = rng.standard_normal(65536) + 1j * rng.standard_normal(65536)
    X = np.fft.fft(x)
    for r in range(4):
        err = np.abs(onepass_bins(x, r) - X[4 * np.arange(16384) + r]).max() / np.abs(X).max()
        assert err < 1e-13, (r, err)
