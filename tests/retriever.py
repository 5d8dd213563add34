"""Client-side digest decode for end-to-end KATs (test infrastructure). Restates
Retriever::decode_digest (retriever.rs:188-260), decode_pertinent_indices (:63-130),
decode_combined_payloads (:318-362) and solve_matrix_mod_257 (matrix.rs:164-247)."""
from __future__ import annotations

import numpy as np

import oracle_lib as O

P = 257


def decrypt_decode(s2, ct) -> np.ndarray:
    """b - a*s in the NTT domain, inverse NTT, round(c*257/q) half up, mod 257."""
    phase = O.decrypt_ntt(s2, np.asarray(ct, dtype=np.uint64)).astype(np.uint64)
    q = np.uint64(1125899906826241)
    t = (phase * np.uint64(2 * P) + q) // (np.uint64(2) * q)  # round half up (retriever.rs:84-89)
    return np.where(t >= P, t - P, t).astype(np.uint32)


def decode_indices(s2, idx_cts, rp: dict, pertinent_count: int) -> set[int]:
    found: set[int] = set()
    spb, sps = rp["slots_per_bucket"], rp["slots_per_segment"]
    for ct in idx_cts:
        dec = decrypt_decode(s2, ct)
        for s in range(len(dec) // sps):
            seg = dec[s * sps:(s + 1) * sps]
            for b in range(sps // spb):
                bucket = seg[b * spb:(b + 1) * spb]
                if bucket[-1] == 1:
                    v = 0
                    for d in bucket[:-1][::-1]:
                        v = v * P + int(d)
                    found.add(v)
        if len(found) == pertinent_count:
            break
    return found


INV_257 = [0] + [pow(i, P - 2, P) for i in range(1, P)]


def solve_mod_257(matrix, rhs):
    """Gaussian elimination mod 257 (matrix.rs:164-247): matrix [rows][cols], rhs [rows][612]."""
    A = [list(map(int, r)) for r in matrix]
    B = [list(map(int, r)) for r in rhs]
    rows, cols = len(A), len(A[0])
    for i in range(cols):
        piv = next((j for j in range(i, rows) if A[j][i] % P), None)
        if piv is None:
            raise ValueError("Matrix is not invertible")
        A[i], A[piv] = A[piv], A[i]
        B[i], B[piv] = B[piv], B[i]
        inv = INV_257[A[i][i] % P]
        A[i] = [(x * inv) % P for x in A[i]]
        B[i] = [(x * inv) % P for x in B[i]]
        for j in range(rows):
            if j != i and A[j][i]:
                c = A[j][i]
                A[j] = [(x - c * y) % P for x, y in zip(A[j], A[i])]
                B[j] = [(x - c * y) % P for x, y in zip(B[j], B[i])]
    return [B[i] for i in range(cols)]


def decode_payloads(s2, pay_cts, weights, all_count: int, indices: list[int], combination_count: int,
                    per_ct: int = 2):
    combined = []
    for ct in pay_cts:
        dec = decrypt_decode(s2, ct)
        for j in range(per_ct):
            combined.append(dec[j * 612:(j + 1) * 612].tolist())
    combined = combined[:combination_count]
    W = np.asarray(weights).reshape(-1, all_count)
    matrix = [[int(W[r, i]) for i in indices] for r in range(combination_count)]
    return solve_mod_257(matrix, combined)
