"""Host test double of the device stretch move (lfg_stretch_propose /
lfg_stretch_accept): numpy Philox4x32-10 with the kernels' counter layout.
Used to check the HIP kernels draw-for-draw and to exercise the sampler's
sharding logic on CPU (gloo)."""
import numpy as np

M0, M1 = np.uint64(0xD2511F53), np.uint64(0xCD9E8D57)
W0, W1 = np.uint64(0x9E3779B9), np.uint64(0xBB67AE85)
MASK = np.uint64(0xFFFFFFFF)


def philox(c0, c1, c2, c3, k0, k1):
    c0, c1, c2, c3 = (np.asarray(c, np.uint64) & MASK for c in (c0, c1, c2, c3))
    k0, k1 = np.uint64(k0) & MASK, np.uint64(k1) & MASK
    for _ in range(10):
        p0 = c0 * M0
        p1 = c2 * M1
        lo0, hi0 = p0 & MASK, p0 >> np.uint64(32)
        lo1, hi1 = p1 & MASK, p1 >> np.uint64(32)
        c0, c1, c2, c3 = (hi1 ^ c1 ^ k0) & MASK, lo1, (hi0 ^ c3 ^ k1) & MASK, lo0
        k0 = (k0 + W0) & MASK
        k1 = (k1 + W1) & MASK
    return c0, c1, c2, c3


def u53(a, b):
    return ((a >> np.uint64(5)) * np.uint64(1 << 26) + (b >> np.uint64(6))).astype(np.float64) / 9007199254740992.0


def draw(seed, step, half, purpose, n):
    i = np.arange(n, dtype=np.uint64)
    return philox(i, np.uint64(step) & MASK, np.uint64(step) >> np.uint64(32),
                  np.uint64(half * 2 + purpose), np.uint64(seed) & MASK, np.uint64(seed) >> np.uint64(32))


def propose(pos, half, a, seed, step):
    W, ndim = pos.shape
    ns = W // 2
    r = draw(seed, step, half, 0, ns)
    u = u53(r[0], r[1])
    z = ((a - 1.0) * u + 1.0) ** 2 / a
    j = ((r[2] * np.uint64(ns)) >> np.uint64(32)).astype(np.int64)
    s = pos[half * ns:(half + 1) * ns]
    c = pos[(1 - half) * ns:(2 - half) * ns][j]
    return c - (c - s) * z[:, None], (ndim - 1.0) * np.log(z)


def accept(pos, lnp, half, q, zfac, lnp_new, seed, step, naccept):
    W = pos.shape[0]
    ns = W // 2
    r = draw(seed, step, half, 1, ns)
    lu = np.log(u53(r[0], r[1]))
    sl = slice(half * ns, (half + 1) * ns)
    with np.errstate(invalid="ignore"):
        acc = lu < zfac + lnp_new - lnp[sl]
    pos[sl][acc] = q[acc]
    lnp[sl][acc] = lnp_new[acc]
    naccept[sl][acc] += 1
    return acc


class TorchCpuOps:
    """EnsembleSampler ops on CPU tensors, via the numpy double."""

    def propose(self, pos, half, a, seed, step, q, zfac):
        import torch
        qq, zz = propose(pos.numpy(), half, a, seed, step)
        q.copy_(torch.as_tensor(qq))
        zfac.copy_(torch.as_tensor(zz))

    def accept(self, pos, lnp, half, q, zfac, lnp_new, seed, step, naccept):
        p, l, n = pos.numpy(), lnp.numpy(), naccept.numpy()
        accept(p, l, half, q.numpy(), zfac.numpy(), lnp_new.numpy(), seed, step, n)
