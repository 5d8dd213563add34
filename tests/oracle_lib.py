"""ctypes binding to oracle/liboracle.so — the CPU parity checker (test infrastructure only)."""
from __future__ import annotations

import ctypes as C
import os
import subprocess

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB_PATH = os.path.join(ROOT, "oracle", "liboracle.so")

_u64p = np.ctypeslib.ndpointer(dtype=np.uint64, flags="C_CONTIGUOUS")
_u32p = np.ctypeslib.ndpointer(dtype=np.uint32, flags="C_CONTIGUOUS")
_u16p = np.ctypeslib.ndpointer(dtype=np.uint16, flags="C_CONTIGUOUS")
_i64p = np.ctypeslib.ndpointer(dtype=np.int64, flags="C_CONTIGUOUS")
_i8p = np.ctypeslib.ndpointer(dtype=np.int8, flags="C_CONTIGUOUS")
_u8p = np.ctypeslib.ndpointer(dtype=np.uint8, flags="C_CONTIGUOUS")

_lib = None


def build() -> None:
    subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "oracle")], check=True)


def lib():
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        build()
    L = C.CDLL(LIB_PATH)
    sig = {
        "oref_ntt_forward": (None, [C.c_int, _u64p]),
        "oref_ntt_inverse": (None, [C.c_int, _u64p]),
        "oref_decompose": (C.c_int, [C.c_int, C.c_uint64, _i64p]),
        "oref_modswitch_q1_to_qi": (C.c_uint64, [C.c_uint64]),
        "oref_first_level_lut": (None, [_u64p]),
        "oref_second_level_lut": (None, [_u64p]),
        "oref_negacyclic_mul_monomial": (None, [C.c_int, _u64p, C.c_uint32, _u64p]),
        "oref_automorphism": (None, [_u64p, C.c_uint32, _u64p]),
        "oref_chacha_block": (None, [C.c_int, _u32p, C.c_uint64, C.c_uint64, _u32p]),
        "oref_create": (C.c_void_p, [_u32p, _u32p, _u64p, _u64p]),
        "oref_destroy": (None, [C.c_void_p]),
        "oref_extract_clue": (None, [_u16p, _u16p, C.c_int, _u16p, _u16p]),
        "oref_br1": (None, [C.c_void_p, _u16p, C.c_uint16, _u64p]),
        "oref_first_level": (None, [C.c_void_p, _u16p, _u16p, _u32p]),
        "oref_br2": (None, [C.c_void_p, _u32p, _u64p]),
        "oref_trace": (None, [C.c_void_p, _u64p, _u64p]),
        "oref_detect": (None, [C.c_void_p, _u16p, _u16p, _u64p]),
        "oref_detect_batch": (None, [C.c_void_p, _u16p, _u16p, C.c_size_t, _u64p, C.c_int]),
        "oref_bucket": (C.c_uint32, [C.c_uint64, C.c_uint32, C.c_uint64, C.c_uint32]),
        "oref_encode_indices": (None, [_u64p, C.c_size_t, C.c_size_t, C.c_size_t, C.c_uint64, C.c_uint32, _u64p]),
        "oref_encode_payloads": (None, [_u64p, _u16p, C.c_size_t, C.c_size_t, C.c_size_t, _u16p,
                                        C.c_uint32, C.c_uint32, _u64p]),
        "oref_payload_weights": (C.c_uint64, [_u8p, C.c_size_t, _u16p]),
        "oref_decrypt_ntt": (None, [_i8p, _u64p, _u64p]),
        "oref_decode_coeff": (C.c_uint32, [C.c_uint64]),
        "oref_clue_phase": (C.c_uint32, [_u16p, _u16p, C.c_int, _u8p]),
        "oref_keygen_secret": (None, [C.c_uint64, C.c_void_p]),
        "oref_keygen_detection_key": (None, [C.c_void_p, C.c_uint64, _u32p, _u32p, _u64p, _u64p, C.c_int]),
        "oref_gen_clues": (None, [C.c_void_p, C.c_uint64, C.c_uint64, C.c_size_t, _u16p, _u16p, C.c_int]),
    }
    for name, (res, args) in sig.items():
        f = getattr(L, name)
        f.restype = res
        f.argtypes = args
    _lib = L
    return L


class OracleDetector:
    """Oracle context over canonical coefficient-domain keys (include/omr_gpu.h layout)."""

    def __init__(self, bsk1, ksk, bsk2, tk):
        L = lib()
        self._h = L.oref_create(np.ascontiguousarray(bsk1, dtype=np.uint32).reshape(-1),
                                np.ascontiguousarray(ksk, dtype=np.uint32).reshape(-1),
                                np.ascontiguousarray(bsk2, dtype=np.uint64).reshape(-1),
                                np.ascontiguousarray(tk, dtype=np.uint64).reshape(-1))

    def close(self):
        if self._h:
            lib().oref_destroy(self._h)
            self._h = None

    def __del__(self):
        self.close()

    def br1(self, lwe_a, lwe_b):
        out = np.zeros(2 * 1024, dtype=np.uint64)
        lib().oref_br1(self._h, np.ascontiguousarray(lwe_a, dtype=np.uint16), int(lwe_b), out)
        return out.reshape(2, 1024)

    def first_level(self, clue_a, clue_b):
        out = np.zeros(671, dtype=np.uint32)
        lib().oref_first_level(self._h, np.ascontiguousarray(clue_a, dtype=np.uint16),
                               np.ascontiguousarray(clue_b, dtype=np.uint16), out)
        return out

    def br2(self, lwe_int):
        out = np.zeros(2 * 2048, dtype=np.uint64)
        lib().oref_br2(self._h, np.ascontiguousarray(lwe_int, dtype=np.uint32), out)
        return out.reshape(2, 2048)

    def trace(self, rlwe):
        out = np.zeros(2 * 2048, dtype=np.uint64)
        lib().oref_trace(self._h, np.ascontiguousarray(rlwe, dtype=np.uint64).reshape(-1), out)
        return out.reshape(2, 2048)

    def detect(self, clue_a, clue_b):
        out = np.zeros(2 * 2048, dtype=np.uint64)
        lib().oref_detect(self._h, np.ascontiguousarray(clue_a, dtype=np.uint16),
                          np.ascontiguousarray(clue_b, dtype=np.uint16), out)
        return out.reshape(2, 2048)

    def detect_batch(self, clue_a, clue_b, nthreads=0):
        D = clue_a.shape[0]
        out = np.zeros(D * 2 * 2048, dtype=np.uint64)
        lib().oref_detect_batch(self._h, np.ascontiguousarray(clue_a, dtype=np.uint16).reshape(-1),
                                np.ascontiguousarray(clue_b, dtype=np.uint16).reshape(-1), D, out, int(nthreads))
        return out.reshape(D, 2, 2048)


class SecretPack(C.Structure):
    """oref_secret_pack (key_gen/secret.rs:46-107 restated in oracle/omr_oracle_keygen.c)."""
    _fields_ = [("s0", C.c_uint8 * 512), ("s1", C.c_int8 * 1024), ("s_int", C.c_uint8 * 670),
                ("s2", C.c_int8 * 2048), ("pk_a", C.c_uint16 * 512), ("pk_b", C.c_uint16 * 512)]

    @classmethod
    def generate(cls, seed: int) -> "SecretPack":
        sk = cls()
        lib().oref_keygen_secret(seed, C.byref(sk))
        return sk

    def export(self):
        return dict(s0=np.ctypeslib.as_array(self.s0).copy(), s1=np.ctypeslib.as_array(self.s1).copy(),
                    s_int=np.ctypeslib.as_array(self.s_int).copy(), s2=np.ctypeslib.as_array(self.s2).copy())

    def generate_detection_key(self, seed: int, nthreads: int = 8):
        """(bsk1, ksk, bsk2, trace_key) in the include/omr_gpu.h layout."""
        bsk1 = np.empty((512, 8, 2, 1024), np.uint32)
        ksk = np.empty((1024, 27, 671), np.uint32)
        bsk2 = np.empty((670, 12, 2, 2048), np.uint64)
        tk = np.empty((11, 25, 2, 2048), np.uint64)
        lib().oref_keygen_detection_key(C.byref(self), seed, bsk1.reshape(-1), ksk.reshape(-1), bsk2.reshape(-1),
                                        tk.reshape(-1), nthreads)
        return bsk1, ksk, bsk2, tk

    def gen_clues(self, seed: int, first: int, count: int, nthreads: int = 8):
        a = np.empty((count, 512), np.uint16)
        b = np.empty((count, 7), np.uint16)
        lib().oref_gen_clues(C.byref(self), seed, first, count, a.reshape(-1), b.reshape(-1), nthreads)
        return a, b


def ntt(level, a):
    a = np.array(a, dtype=np.uint64)
    lib().oref_ntt_forward(level, a)
    return a


def intt(level, a):
    a = np.array(a, dtype=np.uint64)
    lib().oref_ntt_inverse(level, a)
    return a


def decrypt_ntt(s2, ct):
    out = np.zeros(2048, dtype=np.uint64)
    lib().oref_decrypt_ntt(np.ascontiguousarray(s2, dtype=np.int8), np.ascontiguousarray(ct, dtype=np.uint64).reshape(-1), out)
    return out


def decode(c) -> np.ndarray:
    L = lib()
    return np.array([L.oref_decode_coeff(int(x)) for x in np.asarray(c).reshape(-1)], dtype=np.uint32)


def encode_indices(pv, offset, all_count, seed, ct):
    D = pv.shape[0]
    out = np.zeros(2 * 2048, dtype=np.uint64)
    lib().oref_encode_indices(np.ascontiguousarray(pv, dtype=np.uint64).reshape(-1), D, offset, all_count,
                              int(seed), int(ct), out)
    return out.reshape(2, 2048)


def payload_weights(seed: bytes, count: int):
    out = np.zeros(count, dtype=np.uint16)
    rej = lib().oref_payload_weights(np.frombuffer(bytes(seed), dtype=np.uint8).copy(), count, out)
    return out, rej


def encode_payloads(pv, payloads, offset, all_count, weights, n_ct, per_ct):
    D = pv.shape[0]
    out = np.zeros(n_ct * 2 * 2048, dtype=np.uint64)
    lib().oref_encode_payloads(np.ascontiguousarray(pv, dtype=np.uint64).reshape(-1),
                               np.ascontiguousarray(payloads, dtype=np.uint16).reshape(-1), D, offset, all_count,
                               np.ascontiguousarray(weights, dtype=np.uint16), n_ct, per_ct, out)
    return out.reshape(n_ct, 2, 2048)
