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


class Fft8P(Fft):
    """The kernel's level-1 transform (WgFft<64, 8, 9>): passes of 3, 2, 3, 1 stages; the relayouts
    P0 -> P1 and P2 -> P3 are permlane bit swaps (register/lane bits), P1 -> P2 one LDS exchange.
    jidx(p, e) is the transform index held by register e of each lane in pass p."""

    def __init__(self):
        super().__init__(64, 8, 9)

    def jidx(self, p, e):
        l = self.lane
        b = lambda v, k: (v >> k) & 1
        if p == 0:
            return (e << 6) | l
        if p == 1:
            return (b(l, 5) << 8) | (b(l, 4) << 7) | (b(e, 0) << 6) | (b(e, 2) << 5) | (b(e, 1) << 4) | (l & 15)
        if p == 2:
            return ((l & 31) << 4) | (e << 1) | b(l, 5)
        return ((l & 31) << 4) | (b(l, 5) << 3) | (b(e, 1) << 2) | (b(e, 0) << 1) | b(e, 2)

    def relayout(self, x, pf, pt):
        buf = np.full(self.n, np.nan, dtype=np.complex128)
        for e in range(8):
            buf[self.jidx(pf, e)] = x[:, e]
        return np.stack([buf[self.jidx(pt, e)] for e in range(8)], axis=1)

    def blocks(self, p):
        """per-lane premultiplication twiddles of pass p's blocks"""
        tw, l = self.tw, self.lane
        if p in (0, 2):
            hi = 0 if p == 0 else l & 31
            s0 = 0 if p == 0 else 5
            A, B, C = tw[(1 << s0) + hi], tw[(2 << s0) + 2 * hi], tw[(4 << s0) + 4 * hi]
            return [np.ones(64) * v for v in (1, C, B, B * C, A, A * C, A * B, A * B * C)]
        if p == 1:  # two radix-4 blocks (register bit 0 = j6): T = (1, B, A, AB) on registers (e0, e0|2, e0|4, e0|6)
            out = []
            for e0 in (0, 1):
                blk = ((l >> 5) << 2) | (((l >> 4) & 1) << 1) | e0
                A, B = tw[8 + blk], tw[16 + 2 * blk]
                out.append([np.ones(64), B, A, A * B])
            return out
        node = ((l & 31) << 3) | ((l >> 5) << 2)  # stage 8, even node for e1 = 0 (+2 for e1 = 1)
        return [tw[256 + node], tw[256 + node + 2]]

    @staticmethod
    def net8(x):
        P = [x[:, e] for e in range(8)]
        a = [P[e] + P[e + 4] for e in range(4)]
        b = [P[e] - P[e + 4] for e in range(4)]
        c0, c2, c1, c3 = a[0] + a[2], a[0] - a[2], a[1] + a[3], a[1] - a[3]
        d0, d2, d1, d3 = b[0] + 1j * b[2], b[0] - 1j * b[2], b[1] + 1j * b[3], b[1] - 1j * b[3]
        w8 = S8 * (1 + 1j)
        return np.stack([c0 + c1, c0 - c1, c2 + 1j * c3, c2 - 1j * c3, d0 + w8 * d1, d0 - w8 * d1,
                         d2 + 1j * w8 * d3, d2 - 1j * w8 * d3], axis=1)

    @staticmethod
    def net8_adj(x):
        o = [x[:, e] for e in range(8)]
        c0, c1, c2, c3 = o[0] + o[1], o[0] - o[1], o[2] + o[3], -1j * (o[2] - o[3])
        d0, d1 = o[4] + o[5], (1 - 1j) * (o[4] - o[5])
        d2, d3 = o[6] + o[7], (-1 - 1j) * (o[6] - o[7])
        a0, a2, a1, a3 = c0 + c2, c0 - c2, c1 + c3, c1 - c3
        b0, b2, b1, b3 = d0 + d2, -1j * (d0 - d2), d1 + d3, -1j * (d1 - d3)
        return np.stack([a0 + b0, a1 + S8 * b1, a2 + b2, a3 + S8 * b3, a0 - b0, a1 - S8 * b1, a2 - b2,
                         a3 - S8 * b3], axis=1)

    def fwd(self, z):
        x = np.stack([z[self.lane + 64 * e] for e in range(8)], axis=1).astype(np.complex128)
        x = self.net8(x * np.stack(self.blocks(0), axis=1))
        x = self.relayout(x, 0, 1)
        for e0, T in zip((0, 1), self.blocks(1)):
            r = [e0, e0 | 2, e0 | 4, e0 | 6]
            P = [x[:, r[k]] * T[k] for k in range(4)]
            a0, a1, b0, b1 = P[0] + P[2], P[1] + P[3], P[0] - P[2], P[1] - P[3]
            x[:, r[0]], x[:, r[1]], x[:, r[2]], x[:, r[3]] = a0 + a1, a0 - a1, b0 + 1j * b1, b0 - 1j * b1
        x = self.relayout(x, 1, 2)
        x = self.net8(x * np.stack(self.blocks(2), axis=1))
        x = self.relayout(x, 2, 3)
        W = self.blocks(3)
        for e in range(4):  # stage 8 pairs (e, e + 4); register bit 0 = j1 odd siblings take i w
            w = W[(e >> 1) & 1] * (1j if e & 1 else 1)
            u, v = x[:, e].copy(), x[:, e + 4] * w
            x[:, e], x[:, e + 4] = u + v, u - v
        out = np.zeros(self.n, dtype=np.complex128)
        for e in range(8):
            out[self.jidx(3, e)] = x[:, e]
        return out

    def inv(self, X):
        x = np.stack([X[self.jidx(3, e)] for e in range(8)], axis=1).astype(np.complex128)
        W = self.blocks(3)
        for e in range(4):
            w = W[(e >> 1) & 1] * (1j if e & 1 else 1)
            u, v = x[:, e].copy(), x[:, e + 4].copy()
            x[:, e], x[:, e + 4] = u + v, (u - v) * np.conj(w)
        x = self.relayout(x, 3, 2)
        x = self.net8_adj(x) * np.conj(np.stack(self.blocks(2), axis=1))
        x = self.relayout(x, 2, 1)
        for e0, T in zip((0, 1), self.blocks(1)):
            r = [e0, e0 | 2, e0 | 4, e0 | 6]
            o = [x[:, r[k]] for k in range(4)]
            s_, t_, u_, v_ = o[0] + o[1], o[0] - o[1], o[2] + o[3], -1j * (o[2] - o[3])
            P = [s_ + u_, t_ + v_, s_ - u_, t_ - v_]
            for k in range(4):
                x[:, r[k]] = P[k] * np.conj(T[k])
        x = self.relayout(x, 1, 0)
        x = self.net8_adj(x) * np.conj(np.stack(self.blocks(0), axis=1))
        z = np.zeros(self.n, dtype=np.complex128)
        for e in range(8):
            z[self.lane + 64 * e] = x[:, e]
        return z


class Fft8PT(Fft8P):
    """The kernel's level-1 transform since round 5 (device_fft.hpp, WgFft): the same passes and
    layouts as Fft8P, forward butterflies in tangent form (w = c (1 + i t): (p, q) -> (p + c u,
    p - c u), u = q (1 + i t); a factor i of the node applied to c u), the inverse radix-8 passes
    premultiplied as in Fft8P, the inverse P1 / P3 butterflies Gentleman-Sande with
    conj(w) d = c (d (1 - i t))."""

    @staticmethod
    def _ct(w):
        c = np.real(w)
        return c, np.imag(w) / c

    @classmethod
    def bfly(cls, x, a, b, w, odd):
        c, t = cls._ct(w)
        q = x[:, b]
        u = (q.real - t * q.imag) + 1j * (q.imag + t * q.real)
        v = c * u * (1j if odd else 1)
        p = x[:, a].copy()
        x[:, a], x[:, b] = p + v, p - v

    @classmethod
    def ibfly(cls, x, a, b, w, odd):
        c, t = cls._ct(w)
        d = x[:, a] - x[:, b]
        x[:, a] = x[:, a] + x[:, b]
        v = (d.real + t * d.imag) + 1j * (d.imag - t * d.real)
        x[:, b] = c * v * (-1j if odd else 1)

    def nodes8(self, p):
        """per-lane A, B, C, w8 C of pass p's radix-8 block"""
        hi = 0 if p == 0 else self.lane & 31
        s0 = 0 if p == 0 else 5
        tw = self.tw
        return [np.ones(64) * tw[(k << s0) + k * hi + o] for k, o in ((1, 0), (2, 0), (4, 0), (4, 2))]

    def nodes4(self, e0):
        l = self.lane
        blk = ((l >> 5) << 2) | (((l >> 4) & 1) << 1) | e0
        return self.tw[8 + blk], self.tw[16 + 2 * blk]

    def fwd8t(self, x, p):
        A, B, C, W = self.nodes8(p)
        for e in range(4):
            self.bfly(x, e, e + 4, A, False)
        for a, b, odd in ((0, 2, False), (1, 3, False), (4, 6, True), (5, 7, True)):
            self.bfly(x, a, b, B, odd)
        for a, b, w, odd in ((0, 1, C, False), (2, 3, C, True), (4, 5, W, False), (6, 7, W, True)):
            self.bfly(x, a, b, w, odd)

    def fwd(self, z):
        x = np.stack([z[self.lane + 64 * e] for e in range(8)], axis=1).astype(np.complex128)
        self.fwd8t(x, 0)
        x = self.relayout(x, 0, 1)
        for e0 in (0, 1):
            A, B = self.nodes4(e0)
            r0, r1, r2, r3 = e0, e0 | 2, e0 | 4, e0 | 6
            self.bfly(x, r0, r2, A, False)
            self.bfly(x, r1, r3, A, False)
            self.bfly(x, r0, r1, B, False)
            self.bfly(x, r2, r3, B, True)
        x = self.relayout(x, 1, 2)
        self.fwd8t(x, 2)
        x = self.relayout(x, 2, 3)
        W = self.blocks(3)
        for e in range(4):
            self.bfly(x, e, e + 4, W[(e >> 1) & 1], bool(e & 1))
        out = np.zeros(self.n, dtype=np.complex128)
        for e in range(8):
            out[self.jidx(3, e)] = x[:, e]
        return out

    def inv(self, X):
        x = np.stack([X[self.jidx(3, e)] for e in range(8)], axis=1).astype(np.complex128)
        W = self.blocks(3)
        for e in range(4):
            self.ibfly(x, e, e + 4, W[(e >> 1) & 1], bool(e & 1))
        x = self.relayout(x, 3, 2)
        x = self.net8_adj(x) * np.conj(np.stack(self.blocks(2), axis=1))
        x = self.relayout(x, 2, 1)
        for e0 in (0, 1):
            A, B = self.nodes4(e0)
            r0, r1, r2, r3 = e0, e0 | 2, e0 | 4, e0 | 6
            self.ibfly(x, r0, r1, B, False)
            self.ibfly(x, r2, r3, B, True)
            self.ibfly(x, r0, r2, A, False)
            self.ibfly(x, r1, r3, A, False)
        x = self.relayout(x, 1, 0)
        x = self.net8_adj(x) * np.conj(np.stack(self.blocks(0), axis=1))
        z = np.zeros(self.n, dtype=np.complex128)
        for e in range(8):
            z[self.lane + 64 * e] = x[:, e]
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
    ffts = [Fft(*g) for g in geoms] + ([Fft8(*g) for g in geoms] + [Fft8P(), Fft8PT()] if radix8 else [])
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
