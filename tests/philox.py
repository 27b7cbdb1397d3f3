"""numpy restatement of the engine's sampler noise (genie_tts_amd/csrc/common.h):
Philox4x32-10 (Salmon et al. 2011) keyed by the 64-bit seed, counter
(token id, loop step, sequence, 0x51), then Box-Muller on (0,1) uniforms.
The reference draws its N(0,1) from onnxruntime's RandomNormalLike
(stage#1799); ours is this stream -- equal in distribution, not in bits."""
import numpy as np

M0, M1 = np.uint64(0xD2511F53), np.uint64(0xCD9E8D57)
W0, W1 = np.uint32(0x9E3779B9), np.uint32(0xBB67AE85)


def philox4x32(c0, c1, c2, c3, k0, k1):
    c = [np.asarray(v, np.uint32).copy() for v in (c0, c1, c2, c3)]
    k0 = np.uint32(k0)
    k1 = np.uint32(k1)
    for _ in range(10):
        p0 = c[0].astype(np.uint64) * M0
        p1 = c[2].astype(np.uint64) * M1
        hi0, lo0 = (p0 >> np.uint64(32)).astype(np.uint32), p0.astype(np.uint32)
        hi1, lo1 = (p1 >> np.uint64(32)).astype(np.uint32), p1.astype(np.uint32)
        c = [hi1 ^ c[1] ^ k0, lo1, hi0 ^ c[3] ^ k1, lo0]
        k0 = np.uint32((int(k0) + int(W0)) & 0xFFFFFFFF)
        k1 = np.uint32((int(k1) + int(W1)) & 0xFFFFFFFF)
    return c


def u01_open(x):
    """(k + 1/2) / 2^23 of the top 23 bits: exact in f32, strictly inside (0, 1), so q is never +-0."""
    return ((x >> np.uint32(9)).astype(np.float32) + np.float32(0.5)) * np.float32(1.0 / 8388608.0)


def sampler_noise(vocab: int, step: int, b: int, seed: int) -> np.ndarray:
    i = np.arange(vocab, dtype=np.uint32)
    r = philox4x32(i, np.full_like(i, step), np.full_like(i, b), np.full_like(i, 0x51),
                   seed & 0xFFFFFFFF, (seed >> 32) & 0xFFFFFFFF)
    u1, u2 = u01_open(r[0]), u01_open(r[1])
    q = np.sqrt(np.float32(-2.0) * np.log(u1)) * np.cos(np.pi * 2.0 * u2.astype(np.float64)).astype(np.float32)
    return q.astype(np.float32)


def vits_noise(n: int, seed: int) -> np.ndarray:
    """eps of the vocoder's z_p (engine k_noise_philox): element i <- counter (i, 0, 0, 0x7A)."""
    i = np.arange(n, dtype=np.uint32)
    z = np.zeros_like(i)
    r = philox4x32(i, z, z, np.full_like(i, 0x7A), seed & 0xFFFFFFFF, (seed >> 32) & 0xFFFFFFFF)
    u1, u2 = u01_open(r[0]), u01_open(r[1])
    q = np.sqrt(np.float32(-2.0) * np.log(u1)) * np.cos(np.pi * 2.0 * u2.astype(np.float64)).astype(np.float32)
    return q.astype(np.float32)
