"""CPU-side checks of the product library (no GPU): ABI exports, keygen, clues, layout."""
import json
import os
import re

import numpy as np
import pytest

import oracle_lib as O
import product_lib as PL
from product_lib import omr_amd as A

ROOT = PL.ROOT


def test_library_exports_every_declared_symbol():
    hdr = open(os.path.join(ROOT, "include", "omr_gpu.h")).read()
    declared = set(re.findall(r"\b(omr_[a-z0-9_]+)\s*\(", hdr))
    import ctypes
    lib = ctypes.CDLL(A.LIB_PATH)
    missing = [s for s in sorted(declared) if not hasattr(lib, s)]
    assert not missing, missing
    assert declared >= set(A.EXPORTS), "python mirror binds a symbol the header does not declare"


def test_retrieval_params_match_golden():
    prim = json.load(open(os.path.join(ROOT, "tests", "golden", "primitives.json")))
    for D, exp in prim["retrieval"].items():
        rp = A.RetrievalParams(int(D), min(int(D), 50))
        got = {k: getattr(rp, k) for k in exp}
        assert got == exp


def test_payload_weights_match_reference_stream():
    seed = bytes(range(32))
    rp = A.RetrievalParams(64, 10)
    w = A.payload_weights(seed, rp)
    ref, _ = O.payload_weights(seed, rp.combination_count * 64)
    assert np.array_equal(w[: rp.combination_count * 64], ref)
    assert not w[rp.combination_count * 64:].any()
    prim = json.load(open(os.path.join(ROOT, "tests", "golden", "primitives.json")))
    assert w[:300].tolist() == prim["weights"]["values"][:300] or rp.combination_count * 64 < 300


def test_keygen_deterministic_across_thread_counts():
    a = A.SecretKeyPack(3)
    k1 = a.generate_detection_key(11, nthreads=1)
    k2 = a.generate_detection_key(11, nthreads=5)
    for x, y in zip((k1.bsk1, k1.ksk, k1.bsk2, k1.trace_key), (k2.bsk1, k2.ksk, k2.bsk2, k2.trace_key)):
        assert np.array_equal(x, y)
    assert int(k1.bsk1.max()) < A.Q1 and int(k1.bsk2.max()) < A.Q2 and int(k1.ksk.max()) < A.Q1


def test_clues_decrypt_to_zero_under_own_key_only():
    a, b, _ = PL.keys()
    s0 = a.export()["s0"]
    ca, cb = a.gen_clues(5, 100, 16)
    na, nb = b.gen_clues(5, 100, 16)
    L = O.lib()

    def phases(xa, xb):
        p = np.array([[L.oref_clue_phase(xa[m], xb[m], i, s0) for i in range(7)] for m in range(16)])
        return np.where(p > 1024, p - 2048, p)

    own = phases(ca, cb)
    assert np.abs(own).max() < 128  # message 0 within the +-Delta/2 window (Delta = 2048/8)
    other = phases(na, nb)
    assert np.abs(other).max() > 128  # another sender's clues look uniform
    # sharding invariance: clue of global index 103 is the same whichever range produced it
    ca2, cb2 = a.gen_clues(5, 103, 2)
    assert np.array_equal(ca2[0], ca[3]) and np.array_equal(cb2[0], cb[3])


def _build_e2e():
    import subprocess
    subprocess.run(["make", "-s", "-C", os.path.join(PL.ROOT, "tfhe-omr_amd"), "examples"], check=True)
    return os.path.join(PL.ROOT, "tfhe-omr_amd", "build", "omr_e2e")


def test_native_driver_host_only():
    """examples/omr.rs restated in C++ over include/omr_gpu.h compiles against the header, links
    the library and runs its CPU part (keys, clues, weights, retrieval parameters)."""
    import subprocess
    r = subprocess.run([_build_e2e(), "-p", "300", "--host-only"], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr
    assert "5 index ct, 28 payload ct" in r.stdout and "host-only: keys, clues" in r.stdout


def test_on_disk_formats_round_trip(tmp_path):
    """OMRF container (omr_amd.write_arrays): keys, clues and ciphertexts round-trip exactly; a
    wrong kind or a foreign file is rejected."""
    a, _, dk = PL.keys()
    p = str(tmp_path / "dk.omrf")
    A.save_detection_key(p, dk)
    back = A.load_detection_key(p)
    for n in ("bsk1", "ksk", "bsk2", "trace_key"):
        assert np.array_equal(getattr(back, n), getattr(dk, n)) and getattr(back, n).dtype == getattr(dk, n).dtype
    ca, cb = a.gen_clues(3, 100, 17)
    A.save_clues(str(tmp_path / "c.omrf"), ca, cb, first=100)
    la, lb, first = A.load_clues(str(tmp_path / "c.omrf"))
    assert first == 100 and np.array_equal(la, ca) and np.array_equal(lb, cb)
    ct = np.random.default_rng(1).integers(0, A.Q2, (3, 2, 2048), dtype=np.uint64)
    A.save_ciphertexts(str(tmp_path / "ct.omrf"), ct)
    assert np.array_equal(A.load_ciphertexts(str(tmp_path / "ct.omrf")), ct)
    with pytest.raises(A.OmrError):
        A.load_clues(str(tmp_path / "ct.omrf"))
    (tmp_path / "x.bin").write_bytes(b"not a container")
    with pytest.raises(A.OmrError):
        A.load_ciphertexts(str(tmp_path / "x.bin"))


def test_host_keygen_and_clues_match_oracle():
    """The product's host generators (keygen.hip) == the oracle's restatement of
    SecretKeyPack::new / generate_detection_key / ClueKey::gen_clues (oracle/omr_oracle_keygen.c),
    bit for bit, on the same seeded streams: secret keys, every component of the detection key,
    and clues at an offset global index."""
    a, b, dk = PL.keys()
    for pack, seed in ((a, PL.SK_SEED), (b, PL.SK2_SEED)):
        osk = O.SecretPack.generate(seed)
        mine, ref = pack.export(), osk.export()
        for k in ("s0", "s1", "s_int", "s2"):
            assert np.array_equal(mine[k], ref[k]), k
        ha, hb = pack.gen_clues(1000 + seed, 123456, 37)
        oa, ob = osk.gen_clues(1000 + seed, 123456, 37)
        assert np.array_equal(ha, oa) and np.array_equal(hb, ob)
    ref = O.SecretPack.generate(PL.SK_SEED).generate_detection_key(PL.KEY_SEED, nthreads=8)
    for name, x, y in zip(("bsk1", "ksk", "bsk2", "trace_key"), (dk.bsk1, dk.ksk, dk.bsk2, dk.trace_key), ref):
        assert np.array_equal(x, y), name
