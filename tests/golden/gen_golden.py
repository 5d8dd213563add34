"""Generate the golden fixtures under tests/golden/ from the independent Python model
(omr_model.py). Run once; the outputs are committed. Usage:

    python tests/golden/gen_golden.py

Fixtures:
  primitives.json       NTT (by direct evaluation), decomposition, modulus switch, LUTs,
                        retrieval layout, ChaCha (RFC 7539 A.1 #1), payload weights, buckets.
  structured_detect.npz structured-key descriptions + one clue + expected stage outputs.
  encode.npz            small pertinency vector + payloads + expected digests.
"""
from __future__ import annotations

import json
import os
import sys
import time

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
import omr_model as M  # noqa: E402

RFC7539_A1_1 = ("76b8e0ada0f13d90405d6ae55386bd28bdd219b8a08ded1aa836efcc8b770dc7"
                "da41597c5157488d7724e03fb8d84a376a43b8f41518a11cc387b669b2ee6586")


def primitives() -> dict:
    rng = np.random.default_rng(20260227)
    out: dict = {}
    # NTT by definition
    ntt = {}
    for level in (1, 2):
        q, n, _ = M.LEVEL[level]
        vecs = []
        a = [int(x) for x in rng.integers(0, q, n)]
        vecs.append(a)
        delta = [0] * n
        delta[1] = 1  # X -> psi^(2brv(j)+1)
        vecs.append(delta)
        small = [int(x) % q for x in rng.integers(-3, 4, n)]
        vecs.append(small)
        ntt[str(level)] = [{"in": v, "out": M.ntt_direct(level, v)} for v in vecs]
        for v in vecs:
            assert M.ntt_fast(level, v) == M.ntt_direct(level, v)
    out["ntt"] = ntt
    out["psi"] = {"1": M.psi_of(1), "2": M.psi_of(2)}
    # decomposition
    dec = {}
    for which in (1, 2, 3):
        q, logb, d, drop = M.BASIS[which]
        h = (q - 1) // 2
        xs = [0, 1, q - 1, h, h + 1, h - 1, 2, q - 2]
        if drop:
            half = 1 << (drop - 1)
            xs += [half, half - 1, half + 1, q - half, q - half + 1, q - half - 1, 3 * half, q - 3 * half]
        xs += [int(x) for x in rng.integers(0, q, 48)]
        digs = M.decompose_vec(which, np.array(xs, dtype=np.int64))
        dec[str(which)] = {"x": xs, "digits": digs.T.tolist(), "gadget": M.gadget(which)}
    out["decompose"] = dec
    # modulus switch q1 -> 4096
    xs = [0, 1, M.Q1 - 1, M.Q1 // 2, (M.Q1 + 1) // 2] + [int(x) for x in rng.integers(0, M.Q1, 59)]
    out["modswitch"] = {"x": xs, "y": [((2 * M.QI * x + M.Q1) // (2 * M.Q1)) % M.QI for x in xs]}
    # LUTs
    l1, l2 = M.first_level_lut(), M.second_level_lut()
    out["lut1_nonzero"] = [[int(i), int(l1[i])] for i in np.nonzero(l1)[0]]
    out["lut2_nonzero"] = [[int(i), int(l2[i])] for i in np.nonzero(l2)[0]]
    # retrieval layout
    out["retrieval"] = {str(D): M.retrieval_params(D, min(D, 50))
                        for D in (1, 2, 50, 257, 65536, 66049, 66050, 1 << 19, 1 << 20)}
    # ChaCha
    b = M.chacha_block(20, [0] * 8, 0, 0)
    assert "".join(x.to_bytes(4, "little").hex() for x in b) == RFC7539_A1_1
    key = [int(x) for x in rng.integers(0, 1 << 32, 8, dtype=np.uint64)]
    out["chacha"] = {"rfc7539_a1_1": RFC7539_A1_1, "key": key, "counter": 5, "stream": 9,
                     "block12": M.chacha_block(12, key, 5, 9), "block20": M.chacha_block(20, key, 5, 9)}
    seed = bytes(range(32))
    out["weights"] = {"seed": list(seed), "values": M.payload_weights(seed, 300)}
    bk = []
    for (sd, ct, i, s) in [(1, 0, 0, 0), (1, 0, 0, 4), (7, 3, 65535, 2), (123456789, 4, 1000, 6), (2**63 + 5, 7, 2**20 - 1, 1)]:
        bk.append([sd, ct, i, s, M.bucket(sd, ct, i, s)])
    out["buckets"] = bk
    # monomial multiply + automorphism examples
    p = [int(x) for x in rng.integers(0, M.Q2, M.N2)]
    mono = {}
    for r in (0, 1, 2047, 2048, 2049, 4095):
        mono[str(r)] = (M.rot(np.array(p, dtype=np.int64), r) % M.Q2).tolist()
    out["monomial"] = {"p": p, "out": mono}
    auto = {}
    for g in (3, 2049, 1025):
        auto[str(g)] = (M.automorphism(np.array(p, dtype=np.int64), g) % M.Q2).tolist()
    out["automorphism"] = auto
    return out


def structured_detect():
    rng = np.random.default_rng(7)
    s0 = rng.integers(0, 2, M.N0)          # clue LWE key bits (BSK1 messages)
    sint = rng.integers(0, 2, M.NI)        # intermediate LWE key bits (BSK2 messages)
    s1 = M.sparse_secret(rng, M.N1)        # level-1 RLWE secret (sparse ternary)
    s2 = M.sparse_secret(rng, M.N2)        # level-2 RLWE secret
    bsk1 = M.make_structured_bsk(rng, 1, s0, M.N1)
    bsk2 = M.make_structured_bsk(rng, 2, sint, M.N2)
    tk = M.make_structured_trace_key(rng, s2)
    ksk_seed = 99
    ksk = M.ksk_dense(ksk_seed)
    clue_a = rng.integers(0, M.Q0, M.N0)
    clue_b = rng.integers(0, M.Q0, M.CLUES)

    t = time.time()
    la, lb = M.extract_clue(clue_a, clue_b, 0)
    br1_a, br1_b = M.blind_rotate(1, M.first_level_lut(), la, lb, bsk1, s1)
    lwe_int, _ = M.first_level(clue_a, clue_b, bsk1, s1, ksk)
    br2_a, br2_b = M.blind_rotate(2, M.second_level_lut(), lwe_int[:M.NI], int(lwe_int[M.NI]), bsk2, s2)
    tr_a, tr_b = M.trace(br2_a, br2_b, tk, s2)
    print(f"structured detect model: {time.time() - t:.1f}s")

    def ggsw_arrays(keys):
        return (np.array([[list(r) for r in k.alpha] for k in keys], dtype=np.int64),
                np.array([[list(r) for r in k.noise] for k in keys], dtype=np.int64))

    a1, e1 = ggsw_arrays(bsk1)
    a2, e2 = ggsw_arrays(bsk2)
    tka = np.array([[list(r[0]) for r in rows] for (_, _, rows) in tk], dtype=np.int64)
    tke = np.array([[list(r[1]) for r in rows] for (_, _, rows) in tk], dtype=np.int64)
    np.savez_compressed(
        os.path.join(HERE, "structured_detect.npz"),
        s0=s0, sint=sint, s1=np.array(s1, dtype=np.int64), s2=np.array(s2, dtype=np.int64),
        bsk1_alpha=a1, bsk1_noise=e1, bsk2_alpha=a2, bsk2_noise=e2, tk_alpha=tka, tk_noise=tke,
        ksk_seed=np.int64(ksk_seed), clue_a=clue_a.astype(np.uint16), clue_b=clue_b.astype(np.uint16),
        br1_clue0=np.stack([br1_a, br1_b]).astype(np.uint64), lwe_int=lwe_int.astype(np.uint32),
        br2=np.stack([br2_a, br2_b]).astype(np.uint64),
        detect=np.array([tr_a, tr_b], dtype=np.uint64))


def encode():
    rng = np.random.default_rng(11)
    D, offset, all_count = 3, 65533, 65536
    pv = rng.integers(0, M.Q2, (D, 2, M.N2), dtype=np.int64).astype(np.uint64)
    payloads = rng.integers(0, 256, (D, M.PAYLOAD_LEN)).astype(np.uint16)
    seed = 0x1234_5678_9ABC_DEF0
    idx = [M.encode_indices(pv, offset, all_count, seed, ct) for ct in (0, 4)]
    wseed = bytes((i * 7 + 3) & 0xFF for i in range(32))
    n_ct, per_ct = 2, 2
    weights = M.payload_weights(wseed, n_ct * per_ct * all_count)
    pay = M.encode_payloads(pv, payloads, offset, all_count, weights, n_ct, per_ct)
    np.savez_compressed(
        os.path.join(HERE, "encode.npz"),
        pv=pv, payloads=payloads, D=D, offset=offset, all_count=all_count, seed=np.uint64(seed),
        idx_cts=np.array([0, 4]), idx=np.array(idx, dtype=np.uint64), wseed=np.frombuffer(wseed, dtype=np.uint8),
        n_ct=n_ct, per_ct=per_ct, pay=np.array(pay, dtype=np.uint64))


if __name__ == "__main__":
    t0 = time.time()
    with open(os.path.join(HERE, "primitives.json"), "w") as f:
        json.dump(primitives(), f)
    print(f"primitives: {time.time() - t0:.1f}s")
    structured_detect()
    t1 = time.time()
    encode()
    print(f"encode: {time.time() - t1:.1f}s")
