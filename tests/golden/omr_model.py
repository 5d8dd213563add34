"""Independent Python restatement of the InstantOMR detect path, used ONLY to generate and
check golden vectors (test infrastructure; never imported by the product).

It is written without NTTs in the blind rotation / key switch / trace: every external
product is evaluated exactly in the coefficient domain against *structured* evaluation keys
(monomial masks/noise and a sparse ternary secret), so products reduce to signed rotations.
That makes it a genuinely different computation from the C oracle (which uses NTT-domain
keys) while pinning every bit-level convention listed in oracle/omr_oracle.h.

Reference anchors: omr_core/src/detector.rs:135-166 (detect), :457-503 (LUTs), :505-639
(stages), :223-453 (encode), parameters/mod.rs:39-105 (parameters),
parameters/retrieval_params.rs:50-106 (layout), lut.rs:12-27 (negacyclic LUT).
"""
from __future__ import annotations

import numpy as np

# ---------------------------------------------------------------- parameters (mod.rs:39-105)
N0, Q0, CLUES = 512, 2048, 7
Q1, N1, LOGB1, D1, DROP1 = 134215681, 1024, 5, 4, 7
KS_DIGITS, NI, QI, TI = 27, 670, 4096, 32
Q2, N2, LOGB2, D2, DROP2 = 1125899906826241, 2048, 7, 6, 8
LOGBT, DT, TRACE_STEPS = 2, 25, 11
P, PAYLOAD_LEN = 257, 612
G1, G2 = 7, 22  # smallest primitive roots

BASIS = {1: (Q1, LOGB1, D1, DROP1), 2: (Q2, LOGB2, D2, DROP2), 3: (Q2, LOGBT, DT, 0)}
LEVEL = {1: (Q1, N1, G1), 2: (Q2, N2, G2)}


def brv(x: int, bits: int) -> int:
    return int(format(x, f"0{bits}b")[::-1], 2)


def psi_of(level: int) -> int:
    q, n, g = LEVEL[level]
    return pow(g, (q - 1) // (2 * n), q)


# ---------------------------------------------------------------- NTT by definition
def ntt_direct(level: int, a: list[int]) -> list[int]:
    """out[j] = a(psi^(2*brv(j)+1)) — the pinned evaluation order, by direct evaluation."""
    q, n, _ = LEVEL[level]
    L = n.bit_length() - 1
    psi = psi_of(level)
    pw = [pow(psi, k, q) for k in range(2 * n)]
    out = []
    for j in range(n):
        e = 2 * brv(j, L) + 1
        acc = 0
        for i, ai in enumerate(a):
            if ai:
                acc += ai * pw[(e * i) % (2 * n)]
        out.append(acc % q)
    return out


def ntt_fast(level: int, a: list[int]) -> list[int]:
    """Textbook radix-2 CT NTT with python ints (checked against ntt_direct)."""
    q, n, _ = LEVEL[level]
    L = n.bit_length() - 1
    psi = psi_of(level)
    w = [pow(psi, brv(k, L), q) for k in range(n)]
    a = [int(x) % q for x in a]
    m, h = 1, n // 2
    while m < n:
        for i in range(m):
            W = w[m + i]
            for j in range(2 * i * h, 2 * i * h + h):
                U, V = a[j], a[j + h] * W % q
                a[j], a[j + h] = (U + V) % q, (U - V) % q
        m, h = m * 2, h // 2
    return a


# ---------------------------------------------------------------- decomposition
def decompose_vec(which: int, x: np.ndarray) -> np.ndarray:
    """Signed approximate gadget decomposition, digits [d, len(x)] int64 (oracle header)."""
    q, logb, d, drop = BASIS[which]
    x = np.asarray(x, dtype=np.int64)
    y = np.where(x > (q - 1) // 2, x - q, x)
    if drop:
        y = (y + (1 << (drop - 1))) >> drop
    B = 1 << logb
    out = np.empty((d,) + x.shape, dtype=np.int64)
    for k in range(d - 1):
        c = (y + B // 2) >> logb
        out[k] = y - c * B
        y = c
    out[d - 1] = y
    return out


def gadget(which: int) -> list[int]:
    q, logb, d, drop = BASIS[which]
    return [1 << (drop + k * logb) for k in range(d)]


# ---------------------------------------------------------------- polynomial helpers
def rot(p: np.ndarray, r: int) -> np.ndarray:
    """X^r * p in Z[X]/(X^N+1) (no reduction), r any integer."""
    n = p.shape[-1]
    r %= 2 * n
    sign = 1
    if r >= n:
        r -= n
        sign = -1
    if r == 0:
        return sign * p
    return sign * np.concatenate([-p[n - r:], p[: n - r]])


def sparse_mul(p: np.ndarray, sp: list[tuple[int, int]]) -> np.ndarray:
    """p * sum(c * X^t) without reduction (caller keeps magnitudes < 2^63)."""
    out = np.zeros_like(p)
    for c, t in sp:
        out = out + c * rot(p, t)
    return out


def sparse_sparse(a: list[tuple[int, int]], b: list[tuple[int, int]], n: int):
    """product of two sparse polys as a sparse list with negacyclic wrap."""
    acc: dict[int, int] = {}
    for ca, ta in a:
        for cb, tb in b:
            e = (ta + tb) % (2 * n)
            c = ca * cb
            if e >= n:
                e -= n
                c = -c
            acc[e] = acc.get(e, 0) + c
    return [(c, e) for e, c in acc.items() if c]


def sparse_auto(sp: list[tuple[int, int]], g: int, n: int):
    out = []
    for c, t in sp:
        e = (t * g) % (2 * n)
        if e >= n:
            out.append((-c, e - n))
        else:
            out.append((c, e))
    return out


def automorphism(p: np.ndarray, g: int) -> np.ndarray:
    n = p.shape[-1]
    out = np.zeros_like(p)
    e = (np.arange(n, dtype=np.int64) * g) % (2 * n)
    lo = e < n
    out[e[lo]] = p[lo]
    out[e[~lo] - n] = -p[~lo]
    return out


# ---------------------------------------------------------------- LUTs (detector.rs:457-503)
def negacyclic_lut(vals: list[int], n: int, log_t: int) -> np.ndarray:
    hd = n >> log_t
    seq = []
    it1, it2 = list(vals), list(vals[1:])
    for k in range(max(len(it1), len(it2))):  # itertools::interleave
        if k < len(it1):
            seq.append(it1[k])
        if k < len(it2):
            seq.append(it2[k])
    lut = np.zeros(n, dtype=np.int64)
    for c in range(n // hd):
        lut[c * hd:(c + 1) * hd] = seq[c]
    return lut


def first_level_lut() -> np.ndarray:
    log = (32).bit_length() - 1 - 1
    one = ((Q1 >> log) + 1) >> 1
    return negacyclic_lut([one, 0, 0, 0, Q1 - one], N1, 3)


def second_level_lut() -> np.ndarray:
    # BigDecimal(q) / 257 rounded HalfUp
    one = (2 * Q2 + P) // (2 * P)
    data = [0] * TI
    data[2 * CLUES] = one
    return negacyclic_lut(data, N2, 5)


# ---------------------------------------------------------------- structured keys
class StructuredGGSW:
    """GGSW(m) with monomial masks alpha_r = ca*X^ta and monomial noise e_r = ce*X^te."""

    def __init__(self, which: int, m: int, alpha, noise):
        self.which, self.m = which, m
        self.alpha = alpha  # list of (c, t) per row (2d rows)
        self.noise = noise


def make_structured_bsk(rng, which: int, bits, n_poly: int):
    q, logb, d, drop = BASIS[which]
    keys = []
    for m in bits:
        alpha = [(int(rng.integers(1, 1024)), int(rng.integers(0, n_poly))) for _ in range(2 * d)]
        noise = [(int(rng.integers(-8, 9)), int(rng.integers(0, n_poly))) for _ in range(2 * d)]
        keys.append(StructuredGGSW(which, int(m), alpha, noise))
    return keys


def sparse_secret(rng, n: int, h: int = 4):
    pos = rng.choice(n, size=h, replace=False)
    return [(int(rng.choice([-1, 1])), int(t)) for t in pos]


def ext_product(which: int, ta: np.ndarray, tb: np.ndarray, ggsw: StructuredGGSW, s_sparse):
    q, logb, d, drop = BASIS[which]
    n = ta.shape[-1]
    g = gadget(which)
    da = decompose_vec(which, ta)
    db = decompose_vec(which, tb)
    out_a = np.zeros(n, dtype=np.int64)
    out_b = np.zeros(n, dtype=np.int64)
    for r in range(2 * d):
        dig = da[r] if r < d else db[r - d]
        ca, tA = ggsw.alpha[r]
        ce, tE = ggsw.noise[r]
        t = ca * rot(dig, tA)  # dig * alpha_r
        out_a += t
        out_b += sparse_mul(t, s_sparse) + ce * rot(dig, tE)
        if ggsw.m:
            if r < d:
                out_a += g[r] * dig
            else:
                out_b += g[r - d] * dig
        out_a %= q
        out_b %= q
    return out_a, out_b


def blind_rotate(which: int, lut: np.ndarray, lwe_a, lwe_b: int, keys, s_sparse):
    q = BASIS[which][0]
    n = lut.shape[0]
    acc_a = np.zeros(n, dtype=np.int64)
    acc_b = rot(lut, -int(lwe_b)) % q
    for i, ai in enumerate(lwe_a):
        ai = int(ai) % (2 * n)
        if ai == 0:
            continue
        ta = (rot(acc_a, ai) - acc_a) % q
        tb = (rot(acc_b, ai) - acc_b) % q
        ra, rb = ext_product(which, ta, tb, keys[i], s_sparse)
        acc_a = (acc_a + ra) % q
        acc_b = (acc_b + rb) % q
    return acc_a, acc_b


def extract_clue(clue_a, clue_b, i: int):
    a = np.empty(N0, dtype=np.int64)
    for j in range(N0):
        a[j] = clue_a[i - j] if j <= i else (Q0 - int(clue_a[N0 + i - j])) % Q0
    return a, int(clue_b[i]) % Q0


def ksk_dense(seed: int) -> np.ndarray:
    """Deterministic dense KSK [1024*27, 671] mod q1 from a splitmix64-style counter hash."""
    with np.errstate(over="ignore"):
        x = np.arange(N1 * KS_DIGITS * (NI + 1), dtype=np.uint64) + np.uint64(seed) * np.uint64(0x9E3779B97F4A7C15)
        x = x * np.uint64(0xBF58476D1CE4E5B9)
        x ^= x >> np.uint64(31)
        x = x * np.uint64(0x94D049BB133111EB)
        x ^= x >> np.uint64(29)
    return (x % np.uint64(Q1)).astype(np.int64).reshape(N1 * KS_DIGITS, NI + 1)


def first_level(clue_a, clue_b, bsk1, s1_sparse, ksk):
    lut = first_level_lut()
    sa = np.zeros(N1, dtype=np.int64)
    sb = np.zeros(N1, dtype=np.int64)
    for c in range(CLUES):
        la, lb = extract_clue(clue_a, clue_b, c)
        ra, rb = blind_rotate(1, lut, la, lb, bsk1, s1_sparse)
        sa = (sa + ra) % Q1
        sb = (sb + rb) % Q1
    ea = np.empty(N1, dtype=np.int64)
    ea[0] = sa[0]
    ea[1:] = (-sa[N1 - np.arange(1, N1)]) % Q1
    eb = int(sb[0])
    bits = ((ea[:, None] >> np.arange(KS_DIGITS)[None, :]) & 1).reshape(-1)
    sel = ksk[bits.astype(bool)]
    tot = sel.sum(axis=0) % Q1 if sel.shape[0] else np.zeros(NI + 1, dtype=np.int64)
    ka = (-tot[:NI]) % Q1
    kb = (eb - int(tot[NI])) % Q1
    ms = lambda v: ((2 * QI * int(v) + Q1) // (2 * Q1)) % QI  # noqa: E731
    out = np.array([ms(v) for v in ka] + [(ms(kb) + CLUES * (QI // TI)) % QI], dtype=np.int64)
    return out, (sa, sb)


def make_structured_trace_key(rng, s2_sparse):
    keys = []
    for k in range(TRACE_STEPS):
        g = (N2 >> k) + 1
        sg = sparse_auto(s2_sparse, g, N2)
        rows = []
        for j in range(DT):
            alpha = (int(rng.integers(1, 1024)), int(rng.integers(0, N2)))
            noise = (int(rng.integers(-8, 9)), int(rng.integers(0, N2)))
            rows.append((alpha, noise))
        keys.append((g, sg, rows))
    return keys


def trace(rlwe_a, rlwe_b, tkeys, s2_sparse):
    ninv = pow(N2, Q2 - 2, Q2)
    a = np.array([int(x) * ninv % Q2 for x in rlwe_a], dtype=np.int64)
    b = np.array([int(x) * ninv % Q2 for x in rlwe_b], dtype=np.int64)
    for g, sg, rows in tkeys:
        sa = automorphism(a, g) % Q2
        sb = automorphism(b, g) % Q2
        dig = decompose_vec(3, sa)
        A = np.zeros(N2, dtype=np.int64)
        B = np.zeros(N2, dtype=np.int64)
        for j in range(DT):
            (ca, ta), (ce, te) = rows[j]
            t = ca * rot(dig[j], ta)
            A = (A + t) % Q2
            corr = sparse_mul(dig[j], sg)  # dig * sigma_g(s), small
            B = (B + sparse_mul(t, s2_sparse) + ce * rot(dig[j], te) - (1 << (2 * j)) * corr) % Q2
        a = (a + A) % Q2
        b = (b + sb + B) % Q2
    return ntt_fast(2, [int(x) for x in a]), ntt_fast(2, [int(x) for x in b])


# ---------------------------------------------------------------- dense key builders (tests)
def dense_bsk(which: int, keys, s_sparse) -> np.ndarray:
    """Canonical coefficient-domain BSK [n][2d][2][N] (uint64) for structured GGSWs."""
    q, logb, d, drop = BASIS[which]
    n = N1 if which == 1 else N2
    g = gadget(which)
    out = np.zeros((len(keys), 2 * d, 2, n), dtype=np.int64)
    for i, k in enumerate(keys):
        for r in range(2 * d):
            ca, ta = k.alpha[r]
            ce, te = k.noise[r]
            out[i, r, 0, ta] += ca
            for c, e in sparse_sparse([(ca, ta)], s_sparse, n) + [(ce, te)]:
                out[i, r, 1, e] += c
            if k.m:
                out[i, r, 0 if r < d else 1, 0] += g[r if r < d else r - d]
    return (out % q).astype(np.uint64)


def dense_trace_key(tkeys, s2_sparse) -> np.ndarray:
    res = np.zeros((TRACE_STEPS, DT, 2, N2), dtype=np.int64)
    for k, (g, sg, rows) in enumerate(tkeys):
        for j, ((ca, ta), (ce, te)) in enumerate(rows):
            res[k, j, 0, ta] += ca
            for c, e in sparse_sparse([(ca, ta)], s2_sparse, N2) + [(ce, te)]:
                res[k, j, 1, e] += c
            for c, e in sg:
                res[k, j, 1, e] = (res[k, j, 1, e] - c * (1 << (2 * j))) % Q2
    return (res % Q2).astype(np.uint64)


# ---------------------------------------------------------------- ChaCha / rand 0.8 restatement
def chacha_block(rounds: int, key: list[int], counter: int, stream: int) -> list[int]:
    M = 0xFFFFFFFF

    def rl(v, c):
        return ((v << c) | (v >> (32 - c))) & M

    st = [0x61707865, 0x3320646E, 0x79622D32, 0x6B206574] + list(key) + [
        counter & M, (counter >> 32) & M, stream & M, (stream >> 32) & M]
    x = list(st)

    def qr(a, b, c, d):
        x[a] = (x[a] + x[b]) & M; x[d] = rl(x[d] ^ x[a], 16)
        x[c] = (x[c] + x[d]) & M; x[b] = rl(x[b] ^ x[c], 12)
        x[a] = (x[a] + x[b]) & M; x[d] = rl(x[d] ^ x[a], 8)
        x[c] = (x[c] + x[d]) & M; x[b] = rl(x[b] ^ x[c], 7)

    for _ in range(rounds // 2):
        qr(0, 4, 8, 12); qr(1, 5, 9, 13); qr(2, 6, 10, 14); qr(3, 7, 11, 15)
        qr(0, 5, 10, 15); qr(1, 6, 11, 12); qr(2, 7, 8, 13); qr(3, 4, 9, 14)
    return [(x[i] + st[i]) & M for i in range(16)]


def payload_weights(seed: bytes, count: int) -> list[int]:
    """StdRng::from_seed(seed) = ChaCha12 (key=seed, counter 0, stream 0) + rand 0.8
    UniformInt<u16>::sample for [0,257): v:u32, (hi,lo)=v*257, accept lo <= 2^32-2."""
    key = [int.from_bytes(seed[4 * i:4 * i + 4], "little") for i in range(8)]
    out, blk = [], 0
    while len(out) < count:
        for v in chacha_block(12, key, blk, 0):
            m = v * P
            if (m & 0xFFFFFFFF) <= 0xFFFFFFFE:
                out.append(m >> 32)
                if len(out) == count:
                    break
        blk += 1
    return out


def bucket(seed: int, ct: int, i: int, s: int) -> int:
    key = [seed & 0xFFFFFFFF, (seed >> 32) & 0xFFFFFFFF, 0x6F6D7262, ct, 0, 0, 0, 0]
    w = chacha_block(12, key, i, 0x62756B74)
    return (w[s & 15] * 130) >> 32


def retrieval_params(all_count: int, pertinent: int) -> dict:
    pw = 0
    acc = 1
    while acc * P <= all_count:
        acc *= P
        pw += 1
    if acc < all_count:
        pw += 1
    pw = max(pw, 1)
    spb = pw + 1
    sps = spb * 130
    spc = N2 // sps
    cc = pertinent + 5
    return dict(index_slots_per_bucket=pw, slots_per_bucket=spb, slots_per_segment=sps,
                segment_per_cipher=spc, max_encode_indices_cipher_count=25 // spc,
                combination_count=cc, cmb_count_per_cipher=2, cmb_cipher_count=(cc + 1) // 2)


def lift(v: int) -> int:
    return v if v < (P + 1) // 2 else Q2 - P + v


def encode_indices(pv: np.ndarray, offset: int, all_count: int, seed: int, ct: int):
    rp = retrieval_params(all_count, 0)
    out_a = [0] * N2
    out_b = [0] * N2
    for m in range(pv.shape[0]):
        gi = offset + m
        poly = [0] * N2
        for s in range(rp["segment_per_cipher"]):
            bk = bucket(seed, ct, gi, s)
            addr = s * rp["slots_per_segment"] + bk * rp["slots_per_bucket"]
            v, k = gi, 0
            while v:
                dgt = v % P
                poly[addr + k] = lift(dgt)
                v = (v - dgt) // P
                k += 1
            poly[addr + rp["index_slots_per_bucket"]] = 1
        ph = ntt_fast(2, poly)
        for j in range(N2):
            out_a[j] = (out_a[j] + int(pv[m, 0, j]) * ph[j]) % Q2
            out_b[j] = (out_b[j] + int(pv[m, 1, j]) * ph[j]) % Q2
    return out_a, out_b


def encode_payloads(pv, payloads, offset, all_count, weights, n_ct, per_ct):
    outs = []
    for c in range(n_ct):
        oa = [0] * N2
        ob = [0] * N2
        for m in range(pv.shape[0]):
            gi = offset + m
            poly = [0] * N2
            for j in range(per_ct):
                w = weights[(c * per_ct + j) * all_count + gi]
                for l in range(PAYLOAD_LEN):
                    poly[j * PAYLOAD_LEN + l] = lift(int(payloads[m, l]) * w % P)
            ph = ntt_fast(2, poly)
            for j in range(N2):
                oa[j] = (oa[j] + int(pv[m, 0, j]) * ph[j]) % Q2
                ob[j] = (ob[j] + int(pv[m, 1, j]) * ph[j]) % Q2
        outs.append((oa, ob))
    return outs
