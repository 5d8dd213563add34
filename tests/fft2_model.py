"""Lane-exact numpy model of the level-2 complex FFT (tfhe-omr_amd/csrc/br2_fft.hpp, Fft1024):
N2 = 2048 real coefficients folded into n = 1024 complex points z_j = p_j + i p_{j+1024}
(R[X]/(X^2048 + 1) ~ C[X]/(X^1024 - i)), 256 threads x 4 points, five radix-4 passes.

Test infrastructure (tests/test_fft2_layout.py): it restates the device code's index layouts,
twiddle tables, permlane relayouts and LDS exchanges with numpy arrays [thread][register], checks
that forward -> pointwise product -> inverse is the exact negacyclic product, and models the LDS
bank behaviour of every exchange (MI355X_MICROARCH.md, LDS lane groups).

Tree (as the level-1 transform, device_fft.hpp): stage s splits on index bit 9 - s; node i of
stage s has twiddle W(s, i) = w^(eps(s, i) / 2), w = exp(i pi / 2n), eps(0, 0) = n,
eps(s+1, 2i) = eps(s, i) / 2, eps(s+1, 2i+1) = eps(s, i) / 2 + 2n (mod 4n). A radix-4 pass P
(stages 2P, 2P+1) on the block hi (top 2P index bits): registers e = 2 b_hi + b_lo, y = T * x with
T = (1, B, A, AB), A = W(2P, hi), B = W(2P+1, 2 hi); then a0 = y0 + y2, b0 = y0 - y2,
a1 = y1 + y3, b1 = y1 - y3 and out = (a0 + a1, a0 - a1, b0 + i b1, b0 - i b1).
"""
import numpy as np

n, L, T, E = 1024, 10, 256, 4

# Position bits (e1, e0, l5, l4, l3, l2, l1, l0, w1, w0) -> index bit, per pass layout.
LAYOUT = {
    0: (9, 8, 7, 6, 3, 2, 1, 0, 5, 4),
    1: (7, 6, 9, 8, 3, 2, 1, 0, 5, 4),  # P0 -> P1: e1 <-> lane bit 5, e0 <-> lane bit 4 (permlanes)
    2: (5, 4, 3, 2, 1, 0, 9, 8, 7, 6),  # P1 -> P2: cross-wave LDS exchange (X0 / X1)
    3: (3, 2, 5, 4, 1, 0, 9, 8, 7, 6),  # P2 -> P3: permlanes
    4: (1, 0, 5, 4, 3, 2, 9, 8, 7, 6),  # P3 -> P4: wave-local LDS exchange (W); the MAC layout
}


def idx(p, t, e):
    """Point index held by register e of thread t in pass layout p."""
    w, l = t >> 6, t & 63
    bits = ((e >> 1) & 1, e & 1, (l >> 5) & 1, (l >> 4) & 1, (l >> 3) & 1, (l >> 2) & 1, (l >> 1) & 1, l & 1,
            (w >> 1) & 1, w & 1)
    return sum(b << ib for b, ib in zip(bits, LAYOUT[p]))


IDX = {p: np.array([[idx(p, t, e) for e in range(E)] for t in range(T)]) for p in LAYOUT}


def eps_table():
    half = []
    eps = [n]
    for s in range(L):
        half.append([e // 2 for e in eps])
        eps = [x for e in eps for x in ((e // 2) % (4 * n), (e // 2 + 2 * n) % (4 * n))]
    return half  # half[s][i] = eps(s, i) / 2


HALF = eps_table()


def wpow(h):
    return np.exp(1j * np.pi * (h % (8 * n)) / (2 * n))


def block_tw(p, hi):
    """(B, A, AB) of radix-4 pass p, block hi."""
    a, b = HALF[2 * p][hi], HALF[2 * p + 1][2 * hi]
    return wpow(b), wpow(a), wpow(a + b)


def tw_index(p, t):
    """Block (top 2p index bits) of thread t's 4 registers in pass p (the same for all four)."""
    return idx(p, t, 0) >> (L - 2 * p)


# device twiddle table: pass p >= 1 blocks at offset TW_OFF[p] + 3 hi + (0 B, 1 A, 2 AB)
TW_OFF = {1: 0, 2: 3 * 4, 3: 3 * (4 + 16), 4: 3 * (4 + 16 + 64)}
TW_LEN = 3 * (4 + 16 + 64 + 256)


def tw_addr(p, t, k):
    """Global-table (host order) slot (double2) of twiddle k (0 B, 1 A, 2 AB) of thread t's block."""
    return TW_OFF[p] + 3 * tw_index(p, t) + k


def tw_slot(p, b, k):
    """LDS slot of twiddle k of block b (Fft1024::tw_slot): passes 3 and 4 keep each k in its own
    array with the block XOR-swizzled."""
    if p == 3:
        return TW_OFF[3] + k * 64 + (b ^ (((b >> 4) & 3) << 1))
    if p == 4:
        return TW_OFF[4] + k * 256 + (b ^ (((b >> 6) & 3) << 2))
    return TW_OFF[p] + 3 * b + k


def tw_lds(p, t, k):
    """LDS slot of twiddle k of thread t's block in pass p."""
    return tw_slot(p, tw_index(p, t), k)


def twiddle_table():
    tab = np.zeros(TW_LEN, np.complex128)
    for p in range(1, 5):
        for hi in range(4 ** p):
            tab[TW_OFF[p] + 3 * hi: TW_OFF[p] + 3 * hi + 3] = block_tw(p, hi)
    return tab


def fwd_pass(x, p):
    out = np.empty_like(x)
    for t in range(T):
        B, A, AB = block_tw(p, tw_index(p, t))
        y = x[t] * np.array([1, B, A, AB])
        a0, b0, a1, b1 = y[0] + y[2], y[0] - y[2], y[1] + y[3], y[1] - y[3]
        out[t] = (a0 + a1, a0 - a1, b0 + 1j * b1, b0 - 1j * b1)
    return out


def fwd_pass_t(x, p):
    """fwd_pass in the kernel's tangent form since round 5 (Fft1024::fwd_pass_t): A = c_A (1 + i t_A)
    on the pairs (0, 2), (1, 3), then B on (0, 1) and i B on (2, 3), each butterfly
    (p, q) -> (p + c u, p - c u), u = q (1 + i t)."""
    def bf(y, a, b, w, odd):
        c, t = w.real, w.imag / w.real
        q = y[:, b]
        u = (q.real - t * q.imag) + 1j * (q.imag + t * q.real)
        v = c * u * (1j if odd else 1)
        pa = y[:, a].copy()
        y[:, a], y[:, b] = pa + v, pa - v
    y = np.array(x, np.complex128)
    blocks = np.array([tw_index(p, t) for t in range(T)])
    tw = np.array([block_tw(p, b) for b in range(4 ** p)])  # (B, A, AB) per block
    B, A = tw[blocks, 0], tw[blocks, 1]
    bf(y, 0, 2, A, False)
    bf(y, 1, 3, A, False)
    bf(y, 0, 1, B, False)
    bf(y, 2, 3, B, True)
    return y


def inv_pass(x, p):
    """Unscaled inverse of fwd_pass (4 x its inverse)."""
    out = np.empty_like(x)
    for t in range(T):
        B, A, AB = block_tw(p, tw_index(p, t))
        o = x[t]
        a0, a1 = o[0] + o[1], o[0] - o[1]
        b0, b1 = o[2] + o[3], -1j * (o[2] - o[3])
        y = np.array([a0 + b0, a1 + b1, a0 - b0, a1 - b1])
        out[t] = y * np.conj(np.array([1, B, A, AB]))
    return out


def swap_lane_bit(x, ra, rb, lb):
    """Register pair (ra, rb) <-> lane bit lb (v_permlane32_swap lb = 5, v_permlane16_swap lb = 4):
    register ra keeps the lanes with lane bit lb = 0 and receives rb's, rb the other halves."""
    y = x.copy()
    for t in range(T):
        l = t & 63
        if (l >> lb) & 1:
            y[t, ra] = x[t ^ (1 << lb), rb]  # upper lanes of ra <- lower lanes of rb
        else:
            y[t, rb] = x[t ^ (1 << lb), ra]  # lower lanes of rb <- upper lanes of ra
    return y


def relayout_perm(x):
    """P0 <-> P1 and P2 <-> P3: register bit 1 <-> lane bit 5, register bit 0 <-> lane bit 4."""
    x = swap_lane_bit(x, 0, 2, 5)
    x = swap_lane_bit(x, 1, 3, 5)
    x = swap_lane_bit(x, 0, 1, 4)
    x = swap_lane_bit(x, 2, 3, 4)
    return x


def _bit(j, b):
    return (j >> b) & 1


# LDS swizzles of the device exchanges (Fft1024::slot_xf / slot_xi / slot_wf / slot_wi): slot bits
# s0..s9 as XORs of index bits; each is conflict-free in its own direction.
SWIZZLES = {
    "xf": lambda j: _bit(j, 0) | _bit(j, 1) << 1 | (_bit(j, 2) ^ _bit(j, 8)) << 2 | _bit(j, 9) << 3 | _bit(j, 8) << 4
    | _bit(j, 3) << 5 | ((j >> 4) & 15) << 6,
    "xi": lambda j: _bit(j, 0) | (_bit(j, 1) ^ _bit(j, 8)) << 1 | (_bit(j, 2) ^ _bit(j, 9)) << 2 | _bit(j, 3) << 3
    | _bit(j, 8) << 4 | _bit(j, 9) << 5 | ((j >> 4) & 15) << 6,
    "wf": lambda j: _bit(j, 8) | _bit(j, 9) << 1 | (_bit(j, 2) ^ _bit(j, 0)) << 2 | _bit(j, 3) << 3 | _bit(j, 0) << 4
    | _bit(j, 1) << 5 | ((j >> 4) & 15) << 6,
    "wi": lambda j: _bit(j, 8) | _bit(j, 9) << 1 | (_bit(j, 2) ^ _bit(j, 0)) << 2 | _bit(j, 1) << 3 | _bit(j, 0) << 4
    | _bit(j, 3) << 5 | ((j >> 4) & 15) << 6,
}
EXCHANGES = {"xf": (1, 2), "xi": (2, 1), "wf": (3, 4), "wi": (4, 3)}  # swizzle -> (from, to) layout


def slot_stage(c):
    """Rotation staging of 2048 doubles."""
    return c ^ (((c >> 6) & 1) << 4)


# LDS banking (MI355X_MICROARCH.md, LDS): lane groups serviced in one cycle when conflict-free
READ_B128 = [list(range(0, 4)) + list(range(12, 16)) + list(range(20, 28)),
             list(range(4, 12)) + list(range(16, 20)) + list(range(28, 32))]
READ_B128 += [[l + 32 for l in g] for g in READ_B128]
WRITE_B128 = [list(range(8 * i, 8 * i + 8)) for i in range(8)]
READ_B64 = [list(range(0, 32)), list(range(32, 64))]
WRITE_B64 = [list(range(16 * i, 16 * i + 16)) for i in range(4)]


def lds_cycles(addr_bytes, groups, nbanks, width):
    """LDS cycles of one wave instruction: per lane group, the most distinct addresses on a bank."""
    tot = 0
    for g in groups:
        banks = {}
        for l in g:
            a = addr_bytes[l]
            for k in range(width // 4):
                banks.setdefault((a // 4 + k) % nbanks, set()).add(a)
        tot += max(len(v) for v in banks.values())
    return tot


def exchange_cycles(name):
    """(write, read) LDS cycles per instruction of exchange `name`, averaged over waves and registers
    (conflict-free: 8 and 4)."""
    sw, (pf, pt) = SWIZZLES[name], EXCHANGES[name]
    w = r = 0
    for wave in range(4):
        for e in range(E):
            w += lds_cycles([sw(idx(pf, wave * 64 + l, e)) * 16 for l in range(64)], WRITE_B128, 32, 16)
            r += lds_cycles([sw(idx(pt, wave * 64 + l, e)) * 16 for l in range(64)], READ_B128, 64, 16)
    return w / (4 * E), r / (4 * E)


def exchange(x, pf, pt):
    buf = np.zeros(n, x.dtype)
    buf[IDX[pf].ravel()] = x.ravel()
    return buf[IDX[pt]]


def forward(z, tangent=True):
    """z: complex [1024] natural order -> [256][4] spectrum in the P4 (MAC) layout (tangent: the
    kernel's forward passes since round 5; False: the premultiplied passes of rounds 3-4)."""
    fp = fwd_pass_t if tangent else fwd_pass
    x = z[IDX[0]]
    x = fp(x, 0)
    x = relayout_perm(x)
    x = fp(x, 1)
    x = exchange(x, 1, 2)
    x = fp(x, 2)
    x = relayout_perm(x)
    x = fp(x, 3)
    x = exchange(x, 3, 4)
    return fp(x, 4)


def inverse(X):
    """[256][4] in the P4 layout -> complex [1024] natural order, unscaled (x 1024)."""
    x = inv_pass(X, 4)
    x = exchange(x, 4, 3)
    x = inv_pass(x, 3)
    x = relayout_perm(x)
    x = inv_pass(x, 2)
    x = exchange(x, 2, 1)
    x = inv_pass(x, 1)
    x = relayout_perm(x)
    x = inv_pass(x, 0)
    z = np.empty(n, x.dtype)
    z[IDX[0].ravel()] = x.ravel()
    return z


def fold(p):
    return p[:n] + 1j * p[n:]


def unfold(z):
    return np.concatenate([z.real, z.imag])


def negacyclic(a, b):
    """Exact a * b mod (X^2048 + 1) in Python integers."""
    N = len(a)
    full = np.convolve(np.asarray(a, dtype=object), np.asarray(b, dtype=object))
    r = full[:N].copy()
    r[:N - 1] -= full[N:]
    return r


def product(digits_rows, key_rows):
    """sum_r digits_r * key_r mod X^2048 + 1 through the model transform (keys scaled 1/1024):
    the float result before rounding."""
    acc = np.zeros((T, E), np.complex128)
    for d, k in zip(digits_rows, key_rows):
        acc += forward(fold(np.asarray(d, np.float64))) * (forward(fold(np.asarray(k, np.float64))) / n)
    return unfold(inverse(acc))
