"""numpy mirror of rsl_synth_cube's noise (test infrastructure): Philox-4x32-10 (Salmon et al., SC'11) with
key = seed and counter = (global sample index / 2, 0, 0), uint32 -> (x + 1) 2^-32, Box-Muller in fp64."""
import numpy as np

M0, M1 = np.uint64(0xD2511F53), np.uint64(0xCD9E8D57)
W0, W1 = np.uint32(0x9E3779B9), np.uint32(0xBB67AE85)
MASK = np.uint64(0xFFFFFFFF)


def philox4x32_10(c0, c1, c2, c3, k0, k1):
    c0, c1, c2, c3 = (np.asarray(x, dtype=np.uint32) for x in (c0, c1, c2, c3))
    k0, k1 = np.uint32(k0), np.uint32(k1)
    for _ in range(10):
        p0 = M0 * c0.astype(np.uint64)
        p1 = M1 * c2.astype(np.uint64)
        n0 = ((p1 >> np.uint64(32)).astype(np.uint32) ^ c1 ^ k0)
        n1 = (p1 & MASK).astype(np.uint32)
        n2 = ((p0 >> np.uint64(32)).astype(np.uint32) ^ c3 ^ k1)
        n3 = (p0 & MASK).astype(np.uint32)
        c0, c1, c2, c3 = n0, n1, n2, n3
        k0 = np.uint32((int(k0) + int(W0)) & 0xFFFFFFFF)
        k1 = np.uint32((int(k1) + int(W1)) & 0xFFFFFFFF)
    return c0, c1, c2, c3


def noise(shape, seed, frame0=0, noise_power=1.0):
    """complex128 noise of rsl_synth_cube for a cube of `shape` = (F, A, C, S) starting at frame frame0."""
    F, A, C, S = shape
    g0 = frame0 * A * C * S
    npair = F * A * C * S // 2
    q = (np.arange(npair, dtype=np.uint64) * np.uint64(2) + np.uint64(g0)) >> np.uint64(1)
    x0, x1, x2, x3 = philox4x32_10((q & MASK).astype(np.uint32), (q >> np.uint64(32)).astype(np.uint32), 0, 0,
                                   seed & 0xFFFFFFFF, (seed >> 32) & 0xFFFFFFFF)
    u = lambda x: (x.astype(np.float64) + 1.0) * 2.0 ** -32
    sig = np.sqrt(noise_power)
    r0, r1 = sig * np.sqrt(-2 * np.log(u(x0))), sig * np.sqrt(-2 * np.log(u(x2)))
    a0, a1 = 2 * np.pi * u(x1), 2 * np.pi * u(x3)
    out = np.empty(npair * 2, dtype=np.complex128)
    out[0::2] = r0 * np.cos(a0) + 1j * r0 * np.sin(a0)
    out[1::2] = r1 * np.cos(a1) + 1j * r1 * np.sin(a1)
    return out.reshape(shape)
