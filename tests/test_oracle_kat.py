"""The reference's functional KATs on the CPU oracle with real (noisy) keys from the product
keygen: omd.rs:48-58 (detect decrypts to [1,0,..,0] / all zeros) and the end-to-end retrieval
of omr_time_analyze.rs:215-235 (indices and payloads recovered exactly)."""
import numpy as np
import pytest

import oracle_lib as O
import product_lib as PL
import retriever as R
from product_lib import omr_amd as A


@pytest.fixture(scope="module")
def oracle():
    _, _, dk = PL.keys()
    det = O.OracleDetector(dk.bsk1, dk.ksk, dk.bsk2, dk.trace_key)
    yield det
    det.close()


def test_omd_kat(oracle):
    a, _, _ = PL.keys()
    s2 = a.export()["s2"]
    ca, cb = PL.mixed_clues([True, False], seed=77)
    out = oracle.detect_batch(ca, cb, nthreads=2)
    dec = R.decrypt_decode(s2, out[0])
    assert dec[0] == 1 and not dec[1:].any()
    assert not R.decrypt_decode(s2, out[1]).any()


def test_end_to_end_retrieval(oracle):
    a, _, _ = PL.keys()
    s2 = a.export()["s2"]
    D = 6
    mask = np.array([0, 1, 0, 0, 1, 0], dtype=bool)
    ca, cb = PL.mixed_clues(mask, seed=99)
    pv = oracle.detect_batch(ca, cb)
    rng = np.random.default_rng(5)
    payloads = rng.integers(0, 256, (D, 612)).astype(np.uint16)
    rp = A.RetrievalParams(D, int(mask.sum()))
    idx_cts = [O.encode_indices(pv, 0, D, 123, ct) for ct in range(rp.max_encode_indices_cipher_count)]
    found = R.decode_indices(s2, idx_cts, vars(rp), int(mask.sum()))
    assert found == set(np.nonzero(mask)[0].tolist())
    seed = bytes(range(32))
    w = A.payload_weights(seed, rp)
    pay_cts = O.encode_payloads(pv, payloads, 0, D, w, rp.cmb_cipher_count, rp.cmb_count_per_cipher)
    idx = sorted(found)
    solved = R.decode_payloads(s2, pay_cts, w, D, idx, rp.combination_count)
    for i, p in zip(idx, solved):
        assert p == payloads[i].tolist()


def test_native_retriever_matches(oracle):
    """The library's client-side retriever (retriever.hip, Retriever::decode_digest) on oracle
    digests: same plaintexts as the test decoder, exact indices and payloads."""
    a, _, _ = PL.keys()
    s2 = a.export()["s2"]
    D = 5
    mask = np.array([1, 0, 0, 1, 1], dtype=bool)
    ca, cb = PL.mixed_clues(mask, seed=31)
    pv = oracle.detect_batch(ca, cb)
    rng = np.random.default_rng(8)
    payloads = rng.integers(0, 256, (D, 612)).astype(np.uint16)
    rp = A.RetrievalParams(D, int(mask.sum()))
    idx_cts = np.stack([O.encode_indices(pv, 0, D, 7, ct) for ct in range(rp.max_encode_indices_cipher_count)])
    seed = bytes(range(100, 132))
    w = A.payload_weights(seed, rp)
    pay_cts = O.encode_payloads(pv, payloads, 0, D, w, rp.cmb_cipher_count, rp.cmb_count_per_cipher)
    ret = A.Retriever(rp, a)
    for ct in list(idx_cts[:1]) + list(pv[:2]):
        assert np.array_equal(ret.decrypt_decode(ct)[0], R.decrypt_decode(s2, ct))
    indices, pays = ret.decode_digest(idx_cts, pay_cts, seed)
    assert indices == np.nonzero(mask)[0].tolist()
    for i, p in zip(indices, pays):
        assert p.tolist() == payloads[i].tolist()
    # a singular system is reported, not silently solved (OmrError::InvertibleMatrix)
    with pytest.raises(A.OmrError):
        ret.decode_combined_payloads_and_solve(pay_cts, np.zeros_like(w), indices)
