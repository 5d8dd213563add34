"""Model of the level-1 wave FFT (tfhe-omr_amd/csrc/device_fft.hpp), lane by lane: checks that
the twiddle tree, pass indexing and swizzle reproduce the negacyclic product mod X^1024 + 1
exactly after rounding, and reports the worst rounding error (random and adversarial digits)."""
import numpy as np

L, R, E, T = 9, 3, 8, 64
lane = np.arange(T)

def twiddles():
    eps = {(0, 0): 512}
    tw = np.zeros(512, dtype=np.complex128)
    for s in range(9):
        for i in range(1 << s):
            e = eps[(s, i)]
            w_exp = e // 2 if e % 2 == 0 else None
            assert w_exp is not None
            tw[(1 << s) + i] = np.exp(1j * np.pi * np.longdouble(w_exp) / 1024)
            eps[(s + 1, 2 * i)] = (e // 2) % 2048
            eps[(s + 1, 2 * i + 1)] = (e // 2 + 1024) % 2048
    return tw

def index(p, e):
    lb = L - (p + 1) * R
    return ((lane >> lb) << (L - p * R)) | (e << lb) | (lane & ((1 << lb) - 1))

def swz(j):
    return j ^ (((j >> 3) & 1) * 4) ^ (((j >> 4) & 1) * 9) ^ (((j >> 5) & 1) * 15) ^ \
        (((j >> 6) & 1) * 14) ^ (((j >> 8) & 1) * 8)

def exchange(x, pf, pt):
    buf = np.full(512, np.nan, dtype=np.complex128)
    for e in range(E):
        buf[swz(index(pf, e))] = x[:, e]
    assert not np.isnan(buf).any()
    return np.stack([buf[swz(index(pt, e))] for e in range(E)], axis=1)

def fwd_pass(x, P, tw):
    s0, lb = P * R, L - P * R - R
    for k in range(R):
        half = 1 << (R - 1 - k)
        for e in range(E):
            if e & half: continue
            w = tw[(1 << (s0 + k)) + (((lane >> lb) << k) | (e >> (R - k)))]
            v = x[:, e + half] * w
            u = x[:, e].copy()
            x[:, e] = u + v; x[:, e + half] = u - v
    return x

def inv_pass(x, P, tw):
    s0, lb = P * R, L - P * R - R
    for k in range(R - 1, -1, -1):
        half = 1 << (R - 1 - k)
        for e in range(E):
            if e & half: continue
            w = tw[(1 << (s0 + k)) + (((lane >> lb) << k) | (e >> (R - k)))]
            u = x[:, e].copy(); v = x[:, e + half].copy()
            x[:, e] = u + v; x[:, e + half] = (u - v) * np.conj(w)
    return x

def fwd(p, tw):  # p: real length 1024 -> x[lane][e] at transform index 8 lane + e
    z = p[:512] + 1j * p[512:]
    x = np.stack([z[lane + 64 * e] for e in range(E)], axis=1).astype(np.complex128)
    x = fwd_pass(x, 0, tw); x = exchange(x, 0, 1)
    x = fwd_pass(x, 1, tw); x = exchange(x, 1, 2)
    return fwd_pass(x, 2, tw)

def inv(x, tw):
    x = inv_pass(x.copy(), 2, tw); x = exchange(x, 2, 1)
    x = inv_pass(x, 1, tw); x = exchange(x, 1, 0)
    x = inv_pass(x, 0, tw)
    z = np.zeros(512, dtype=np.complex128)
    for e in range(E):
        z[lane + 64 * e] = x[:, e]
    return np.concatenate([z.real, z.imag])

def negacyclic(a, b):
    full = np.convolve(a.astype(object), b.astype(object))
    r = full[:1024].copy(); r[:1023] -= full[1024:]
    return r

def main():
    tw = twiddles()
    rng = np.random.default_rng(5)
    q1 = 134215681
    worst = 0.0
    for trial in range(8):
        keys = [rng.integers(-(q1 - 1) // 2, (q1 - 1) // 2 + 1, 1024) for _ in range(8)]
        if trial % 2 == 0:
            digs = [rng.integers(-16, 18, 1024) for _ in range(8)]
        else:  # adversarial for output coefficient `c`
            c = int(rng.integers(1024)); digs = []
            for k in keys:  # out_c = sum_j d_j * k_{c-j} * sign
                d = np.zeros(1024, dtype=np.int64)
                for j in range(1024):
                    t = c - j; s = 1
                    if t < 0: t += 1024; s = -1
                    d[j] = 17 * s * int(np.sign(k[t]))
                digs.append(d)
        acc = sum(fwd(d.astype(float), tw) * (fwd(k.astype(float), tw) / 512) for d, k in zip(digs, keys))
        out = inv(acc, tw)
        exact = np.array(sum(negacyclic(d, k) for d, k in zip(digs, keys)), dtype=np.float64)
        err = float(np.max(np.abs(out - exact)))
        assert np.array_equal(np.rint(out), exact), "rounding mismatch"
        worst = max(worst, err)
        print(f"trial {trial}: max |coef| {np.max(np.abs(exact)):.3e}  max error {err:.3e}")
    print(f"worst error {worst:.3e} (rounding threshold 0.5)")

if __name__ == "__main__":
    main()
