"""Lane-exact model of the workgroup FFTs (tfhe-omr_amd/csrc/device_fft.hpp): checks that the
twiddle tree, pass indexing and swizzle reproduce the negacyclic product exactly after rounding,
reports the worst rounding error for random and adversarial digits, and checks that geometries
of one size agree on the transform order (keys transformed by one can be used by the other).
Level 1 runs the kernel's radix-8 passes (Fft8: premultiply by T_e, constant 8-point network)
next to the plain radix-2 stages (Fft); level 2 (a 2-limb FFT, not in the product) radix-2 only.
    python tools/fft_exactness.py            # level 1 (64 x 8, N = 1024)
    python tools/fft_exactness.py --level 2  # level 2 (256 x 4 and 64 x 16, N = 2048, 2 limbs)"""
import sys
import numpy as np


class Fft:
    def __init__(self, T, E, L, pair=True):
        self.T, self.E, self.L, self.pair = T, E, L, pair
        self.R = E.bit_length() - 1
        self.NP = (L + self.R - 1) // self.R
        self.n = 1 << L
        self.lane = np.arange(T)
        n = self.n
        eps = {(0, 0): n}
        self.tw = np.zeros(n, dtype=np.complex128)
        for s in range(L):
            for i in range(1 << s):
                e = eps[(s, i)]
                self.tw[(1 << s) + i] = np.exp(1j * np.pi * np.longdouble(e // 2) / (2 * n))
                eps[(s + 1, 2 * i)] = (e // 2) % (4 * n)
                eps[(s + 1, 2 * i + 1)] = (e // 2 + 2 * n) % (4 * n)

    def stages(self, p):
        return min(self.R, self.L - p * self.R)

    def index(self, p, e):
        R, L = self.R, self.L
        s0, r = p * R, self.stages(p)
        lb = L - s0 - r
        F = (self.lane << (R - r)) | (e >> r)
        return ((F >> lb) << (L - s0)) | ((e & ((1 << r) - 1)) << lb) | (F & ((1 << lb) - 1))

    def node(self, p, k, e):
        R, L = self.R, self.L
        s0, r = p * R, self.stages(p)
        lb = L - s0 - r
        F = (self.lane << (R - r)) | (e >> r)
        return (1 << (s0 + k)) + (((F >> lb) << k) | ((e & ((1 << r) - 1)) >> (r - k)))

    def twiddle(self, p, k, e):
        """(w, odd): with pairing (OMR_FFT_TW_PAIR) an odd sibling node reads its even sibling's
        twiddle and the kernel applies the factor i (w_odd = i w_even)."""
        r = self.stages(p)
        pb = (1 << (r - k)) if (self.pair and k >= 1) else 0
        odd = bool(e & pb)
        w = self.tw[self.node(p, k, e & ~pb if odd else e)]
        return w, odd

    def exchange(self, x, pf, pt):
        buf = np.full(self.n, np.nan, dtype=np.complex128)
        for e in range(self.E):
            buf[self.index(pf, e)] = x[:, e]
        assert not np.isnan(buf).any()
        return np.stack([buf[self.index(pt, e)] for e in range(self.E)], axis=1)

    def fwd(self, z):  # z: n complex (folded coefficients) -> x[lane][e] at transform index
        x = np.stack([z[self.lane + self.T * e] for e in range(self.E)], axis=1).astype(np.complex128)
        for p in range(self.NP):
            if p:
                x = self.exchange(x, p - 1, p)
            r = self.stages(p)
            for k in range(r):
                half = 1 << (r - 1 - k)
                for e in range(self.E):
                    if e & half:
                        continue
                    w, odd = self.twiddle(p, k, e)
                    v = x[:, e + half] * w * (1j if odd else 1)
                    u = x[:, e].copy()
                    x[:, e], x[:, e + half] = u + v, u - v
        out = np.zeros(self.n, dtype=np.complex128)
        for e in range(self.E):
            out[self.index(self.NP - 1, e)] = x[:, e]
        return out  # indexed by transform index

    def inv(self, X):
        x = np.stack([X[self.index(self.NP - 1, e)] for e in range(self.E)], axis=1).astype(np.complex128)
        for p in range(self.NP - 1, -1, -1):
            if p < self.NP - 1:
                x = self.exchange(x, p + 1, p)
            r = self.stages(p)
            for k in range(r - 1, -1, -1):
                half = 1 << (r - 1 - k)
                for e in range(self.E):
                    if e & half:
                        continue
                    w, odd = self.twiddle(p, k, e)
                    u, v = x[:, e].copy(), x[:, e + half].copy()
                    x[:, e], x[:, e + half] = u + v, (u - v) * np.conj(w) * (-1j if odd else 1)
        z = np.zeros(self.n, dtype=np.complex128)
        for e in range(self.E):
            z[self.lane + self.T * e] = x[:, e]
        return z


S8 = np.sqrt(0.5)


class Fft8(Fft):
    """Radix-8 passes as in WgFft::fwd_pass / inv_pass (L a multiple of 3)."""

    def block_tw(self, p):
        s0, hi = 3 * p, self.lane >> (self.L - 3 * p - 3)
        A, B, C = self.tw[(1 << s0) + hi], self.tw[(2 << s0) + 2 * hi], self.tw[(4 << s0) + 4 * hi]
        return [1, C, B, B * C, A, A * C, A * B, A * B * C]

    def fwd(self, z):
        x = np.stack([z[self.lane + self.T * e] for e in range(self.E)], axis=1).astype(np.complex128)
        for p in range(self.NP):
            if p:
                x = self.exchange(x, p - 1, p)
            T = self.block_tw(p)
            P = [x[:, e] * T[e] for e in range(8)]
            a = [P[e] + P[e + 4] for e in range(4)]
            b = [P[e] - P[e + 4] for e in range(4)]
            c0, c2, c1, c3 = a[0] + a[2], a[0] - a[2], a[1] + a[3], a[1] - a[3]
            d0, d2, d1, d3 = b[0] + 1j * b[2], b[0] - 1j * b[2], b[1] + 1j * b[3], b[1] - 1j * b[3]
            w8 = S8 * (1 + 1j)
            x = np.stack([c0 + c1, c0 - c1, c2 + 1j * c3, c2 - 1j * c3, d0 + w8 * d1, d0 - w8 * d1,
                          d2 + 1j * w8 * d3, d2 - 1j * w8 * d3], axis=1)
        out = np.zeros(self.n, dtype=np.complex128)
        for e in range(self.E):
            out[self.index(self.NP - 1, e)] = x[:, e]
        return out

    def inv(self, X):
        x = np.stack([X[self.index(self.NP - 1, e)] for e in range(self.E)], axis=1).astype(np.complex128)
        for p in range(self.NP - 1, -1, -1):
            if p < self.NP - 1:
                x = self.exchange(x, p + 1, p)
            T = self.block_tw(p)
            o = [x[:, e] for e in range(8)]
            c0, c1, c2, c3 = o[0] + o[1], o[0] - o[1], o[2] + o[3], -1j * (o[2] - o[3])
            d0, d1 = o[4] + o[5], (1 - 1j) * (o[4] - o[5])
            d2, d3 = o[6] + o[7], (-1 - 1j) * (o[6] - o[7])
            a0, a2, a1, a3 = c0 + c2, c0 - c2, c1 + c3, c1 - c3
            b0, b2, b1, b3 = d0 + d2, -1j * (d0 - d2), d1 + d3, -1j * (d1 - d3)
            P = [a0 + b0, a1 + S8 * b1, a2 + b2, a3 + S8 * b3, a0 - b0, a1 - S8 * b1, a2 - b2, a3 - S8 * b3]
            x = np.stack([P[e] * np.conj(T[e]) for e in range(8)], axis=1)
        z = np.zeros(self.n, dtype=np.complex128)
        for e in range(self.E):
            z[self.lane + self.T * e] = x[:, e]
        return z


def fold(p):
    h = len(p) // 2
    return p[:h] + 1j * p[h:]


def unfold(z):
    return np.concatenate([z.real, z.imag])


def negacyclic(a, b):
    N = len(a)
    full = np.convolve(a.astype(object), b.astype(object))
    r = full[:N].copy()
    r[:N - 1] -= full[N:]
    return r


def adversarial(keys, dmax, N, rng):
    c = int(rng.integers(N))
    out = []
    for k in keys:
        t = (c - np.arange(N)) % N
        sign = np.where(np.arange(N) <= c, 1, -1)
        out.append(dmax * sign * np.sign(k[t]).astype(np.int64))
    return out


def run(geoms, N, kbits, dmax, rows, trials=4, radix8=False):
    rng = np.random.default_rng(5)
    ffts = [Fft(*g) for g in geoms] + ([Fft8(*g) for g in geoms] if radix8 else [])
    worst = 0.0
    for trial in range(trials):
        keys = [rng.integers(-(1 << (kbits - 1)), 1 << (kbits - 1), N) for _ in range(rows)]
        digs = [rng.integers(-dmax, dmax + 1, N) for _ in range(rows)] if trial % 2 == 0 else \
            adversarial(keys, dmax, N, rng)
        exact = np.array(sum(negacyclic(d, k) for d, k in zip(digs, keys)), dtype=np.float64)
        spectra = []
        for f in ffts:
            acc = sum(f.fwd(fold(d.astype(float))) * (f.fwd(fold(k.astype(float))) / (N // 2))
                      for d, k in zip(digs, keys))
            spectra.append(acc)
            out = unfold(f.inv(acc))
            assert np.array_equal(np.rint(out), exact), f"rounding mismatch {f.T}x{f.E}"
            worst = max(worst, float(np.max(np.abs(out - exact))))
        for a in spectra[1:]:  # same transform order across geometries
            assert np.allclose(a, spectra[0], rtol=1e-12, atol=1e-6)
        print(f"trial {trial}: max |coef| {np.max(np.abs(exact)):.3e} worst error so far {worst:.3e}")
    print(f"worst error {worst:.3e} (rounding threshold 0.5)")


if __name__ == "__main__":
    if "--level" in sys.argv and sys.argv[sys.argv.index("--level") + 1] == "2":
        run([(256, 4, 10), (64, 16, 10)], 2048, 25, 64, 12)
    else:
        run([(64, 8, 9)], 1024, 27, 17, 8, trials=8, radix8=True)
