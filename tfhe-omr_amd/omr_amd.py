"""Python host mirror of omr_core's public API over libomr_gpu.so (include/omr_gpu.h).

Names follow the reference (omr_core/src/lib.rs:21-31): KeyGen, SecretKeyPack, DetectionKey,
Detector (detect / detect_with_time_info / encode_pertinent_indices /
encode_pertinent_payloads), RetrievalParams, Payload helpers. Every compute call goes through
the HIP C ABI; there is no CPU fallback: if libomr_gpu.so is missing this module raises.
"""
from __future__ import annotations

import atexit
import ctypes as C
import os
import weakref
from dataclasses import dataclass

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("OMR_GPU_LIB", os.path.join(HERE, "libomr_gpu.so"))

N0, CLUE_COUNT, N1, NI, N2 = 512, 7, 1024, 670, 2048
Q1, Q2, P = 134215681, 1125899906826241, 257
KS_DIGITS, TRACE_STEPS, TRACE_DIGITS, PAYLOAD_LENGTH = 27, 11, 25, 612
BSK1_SHAPE = (N0, 8, 2, N1)
KSK_SHAPE = (N1, KS_DIGITS, NI + 1)
BSK2_SHAPE = (NI, 12, 2, N2)
TK_SHAPE = (TRACE_STEPS, TRACE_DIGITS, 2, N2)

_u64p = np.ctypeslib.ndpointer(dtype=np.uint64, flags="C_CONTIGUOUS")
_u32p = np.ctypeslib.ndpointer(dtype=np.uint32, flags="C_CONTIGUOUS")
_u16p = np.ctypeslib.ndpointer(dtype=np.uint16, flags="C_CONTIGUOUS")
_u8p = np.ctypeslib.ndpointer(dtype=np.uint8, flags="C_CONTIGUOUS")
_i8p = np.ctypeslib.ndpointer(dtype=np.int8, flags="C_CONTIGUOUS")


class OmrError(RuntimeError):
    pass


class _RetrievalParams(C.Structure):
    _fields_ = [(n, C.c_uint32) for n in (
        "index_slots_per_bucket", "slots_per_bucket", "slots_per_segment", "segment_per_cipher",
        "max_encode_indices_cipher_count", "combination_count", "cmb_count_per_cipher", "cmb_cipher_count")]


class _KeyView(C.Structure):
    _fields_ = [("bsk1", C.c_void_p), ("ksk", C.c_void_p), ("bsk2", C.c_void_p), ("trace_key", C.c_void_p)]


class _Timing(C.Structure):
    """omr_detect_timing: DetectTimeInfo (detector.rs:51-57) in milliseconds of device time."""
    _fields_ = [("total_ms", C.c_float), ("first_level_ms", C.c_float), ("second_level_ms", C.c_float),
                ("trace_ms", C.c_float), ("key_switch_ms", C.c_float), ("messages", C.c_size_t),
                ("trace_separate", C.c_int)]


EXPORTS = {
    "omr_last_error": (C.c_char_p, []),
    "omr_version": (C.c_char_p, []),
    "omr_detect_kernels": (C.c_char_p, []),
    "omr_keygen_secret": (C.c_int, [C.c_uint64, C.POINTER(C.c_void_p)]),
    "omr_secret_destroy": (None, [C.c_void_p]),
    "omr_secret_export": (C.c_int, [C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p]),
    "omr_keygen_detection_key": (C.c_int, [C.c_void_p, C.c_uint64, _u32p, _u32p, _u64p, _u64p, C.c_int]),
    "omr_gen_clues": (C.c_int, [C.c_void_p, C.c_uint64, C.c_uint64, C.c_size_t, _u16p, _u16p, C.c_int]),
    "omr_gen_clues_device": (C.c_int, [C.c_void_p, C.c_uint64, C.c_uint64, C.c_size_t, C.c_void_p, C.c_void_p,
                                       C.c_void_p]),
    "omr_keygen_detection_key_device": (C.c_int, [C.c_void_p, C.c_uint64, C.c_void_p, C.c_void_p, C.c_void_p,
                                                  C.c_void_p, C.c_void_p]),
    "omr_get_retrieval_params": (C.c_int, [C.c_size_t, C.c_size_t, C.POINTER(_RetrievalParams)]),
    "omr_payload_weights": (C.c_int, [_u8p, C.c_size_t, C.c_uint32, C.c_uint32, C.c_uint32, _u16p]),
    "omr_ctx_create": (C.c_int, [C.POINTER(_KeyView), C.c_int, C.POINTER(C.c_void_p)]),
    "omr_ctx_destroy": (None, [C.c_void_p]),
    "omr_ctx_set_batch": (C.c_int, [C.c_void_p, C.c_size_t]),
    "omr_ctx_set_latency_threshold": (C.c_int, [C.c_void_p, C.c_size_t]),
    "omr_ctx_set_exact_level1": (C.c_int, [C.c_void_p, C.c_int]),
    "omr_ctx_set_encode_chunks": (C.c_int, [C.c_void_p, C.c_size_t]),
    "omr_detect_batch": (C.c_int, [C.c_void_p, _u16p, _u16p, C.c_size_t, _u64p]),
    "omr_detect": (C.c_int, [C.c_void_p, _u16p, _u16p, _u64p]),
    "omr_ctx_set_coalescing": (C.c_int, [C.c_void_p, C.c_size_t, C.c_long]),
    "omr_ctx_coalescing_stats": (C.c_int, [C.c_void_p, C.POINTER(C.c_size_t), C.POINTER(C.c_size_t)]),
    "omr_detect_batch_device": (C.c_int, [C.c_void_p, C.c_void_p, C.c_void_p, C.c_size_t, C.c_void_p, C.c_void_p]),
    "omr_ctx_enable_timing": (C.c_int, [C.c_void_p, C.c_int]),
    "omr_last_timing": (C.c_int, [C.c_void_p, C.POINTER(_Timing)]),
    "omr_detect_with_time_info": (C.c_int, [C.c_void_p, _u16p, _u16p, C.c_size_t, _u64p, C.POINTER(_Timing)]),
    "omr_ctx_check": (C.c_int, [C.c_void_p, C.c_void_p]),
    "omr_ctx_set_rounding_guard": (C.c_int, [C.c_void_p, C.c_int]),
    "omr_ctx_rounding_margin": (C.c_int, [C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p, C.c_int]),
    "omr_ctx_exactness": (C.c_int, [C.c_void_p, C.c_void_p, C.c_void_p]),
    "omr_fft_twiddles_dd": (C.c_int, [C.c_int, np.ctypeslib.ndpointer(dtype=np.float64, flags="C_CONTIGUOUS")]),
    "omr_ctx_key_spectrum": (C.c_int, [C.c_void_p, C.c_int, C.c_size_t, C.c_size_t,
                                       np.ctypeslib.ndpointer(dtype=np.float64, flags="C_CONTIGUOUS")]),
    "omr_encode_indices": (C.c_int, [C.c_void_p, _u64p, C.c_size_t, C.c_size_t, C.c_size_t, C.c_uint64,
                                     C.c_uint32, _u64p]),
    "omr_encode_indices_device": (C.c_int, [C.c_void_p, C.c_void_p, C.c_size_t, C.c_size_t, C.c_size_t,
                                            C.c_uint64, C.c_uint32, C.c_uint32, C.c_void_p, C.c_void_p]),
    "omr_encode_payloads": (C.c_int, [C.c_void_p, _u64p, _u16p, C.c_size_t, C.c_size_t, C.c_size_t, _u16p,
                                      C.c_uint32, C.c_uint32, _u64p]),
    "omr_encode_payloads_device": (C.c_int, [C.c_void_p, C.c_void_p, C.c_void_p, C.c_size_t, C.c_size_t,
                                             C.c_size_t, C.c_void_p, C.c_uint32, C.c_uint32, C.c_void_p,
                                             C.c_void_p]),
    "omr_first_level": (C.c_int, [C.c_void_p, _u16p, _u16p, C.c_size_t, _u32p]),
    "omr_blind_rotate_level1": (C.c_int, [C.c_void_p, _u16p, _u16p, C.c_size_t, _u64p]),
    "omr_fft1_mul": (C.c_int, [C.c_void_p, _u32p, _u32p, C.c_size_t, _u64p]),
    "omr_decrypt_decode": (C.c_int, [C.c_void_p, _u64p, C.c_size_t, _u32p]),
    "omr_retrieve_indices": (C.c_int, [C.c_void_p, _u64p, C.c_uint32, C.c_size_t, C.c_size_t,
                                       np.ctypeslib.ndpointer(dtype=np.uintp, flags="C_CONTIGUOUS"),
                                       C.c_size_t, C.POINTER(C.c_size_t)]),
    "omr_retrieve_payloads": (C.c_int, [C.c_void_p, _u64p, C.c_uint32, C.c_size_t, C.c_uint32, _u16p,
                                        np.ctypeslib.ndpointer(dtype=np.uintp, flags="C_CONTIGUOUS"),
                                        C.c_size_t, _u16p]),
    "omr_second_level": (C.c_int, [C.c_void_p, _u32p, C.c_size_t, _u64p]),
    "omr_blind_rotate_level2": (C.c_int, [C.c_void_p, _u32p, C.c_size_t, _u64p]),
    "omr_ntt": (C.c_int, [C.c_int, C.c_int, _u64p, C.c_size_t, C.c_int]),
}

_lib = None


def lib():
    """Load libomr_gpu.so (fails loudly: there is no CPU path)."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise OmrError(f"{LIB_PATH} not found: build it with `make -C tfhe-omr_amd` "
                           "(or __graft_entry__.build())")
        L = C.CDLL(LIB_PATH)
        for name, (res, args) in EXPORTS.items():
            f = getattr(L, name)
            f.restype = res
            f.argtypes = args
        _lib = L
    return _lib


def _check(st: int, what: str) -> None:
    if st != 0:
        raise OmrError(f"{what} failed ({st}): {lib().omr_last_error().decode()}")


@dataclass
class RetrievalParams:
    """RetrievalParams::new(257, 2048, all, pertinent, 130, 25, 2) (retrieval_params.rs:50-106)."""
    all_payloads_count: int
    pertinent_count: int
    index_slots_per_bucket: int = 0
    slots_per_bucket: int = 0
    slots_per_segment: int = 0
    segment_per_cipher: int = 0
    max_encode_indices_cipher_count: int = 0
    combination_count: int = 0
    cmb_count_per_cipher: int = 0
    cmb_cipher_count: int = 0

    def __post_init__(self):
        rp = _RetrievalParams()
        _check(lib().omr_get_retrieval_params(self.all_payloads_count, self.pertinent_count, C.byref(rp)),
               "omr_get_retrieval_params")
        for n, _ in _RetrievalParams._fields_:
            setattr(self, n, getattr(rp, n))


def payload_weights(seed: bytes, rp: RetrievalParams) -> np.ndarray:
    """Seeded weights in the reference order (detector.rs:376-387): [n_ct*per_ct][all] u16."""
    n = rp.cmb_cipher_count * rp.cmb_count_per_cipher * rp.all_payloads_count
    out = np.zeros(n, dtype=np.uint16)
    _check(lib().omr_payload_weights(np.frombuffer(bytes(seed), dtype=np.uint8).copy(), rp.all_payloads_count,
                                     rp.combination_count, rp.cmb_cipher_count, rp.cmb_count_per_cipher, out),
           "omr_payload_weights")
    return out


@dataclass
class DetectionKey:
    """Coefficient-domain evaluation keys (key_gen/detection.rs:9-16) in the ABI layout."""
    bsk1: np.ndarray
    ksk: np.ndarray
    bsk2: np.ndarray
    trace_key: np.ndarray

    def size(self) -> int:
        return sum(a.nbytes for a in (self.bsk1, self.ksk, self.bsk2, self.trace_key))


class SecretKeyPack:
    """KeyGen::generate_secret_key / SecretKeyPack (key_gen/secret.rs:46-209), seeded."""

    def __init__(self, seed: int):
        h = C.c_void_p()
        _check(lib().omr_keygen_secret(seed, C.byref(h)), "omr_keygen_secret")
        self._h = h
        self.seed = seed
        # bound now: at interpreter shutdown the module's globals (lib) may already be None
        self._destroy = lib().omr_secret_destroy

    def __del__(self):
        if getattr(self, "_h", None):
            self._destroy(self._h)
            self._h = None

    def export(self):
        s0 = np.zeros(N0, np.uint8)
        s1 = np.zeros(N1, np.int8)
        sint = np.zeros(NI, np.uint8)
        s2 = np.zeros(N2, np.int8)
        _check(lib().omr_secret_export(self._h, s0.ctypes.data, s1.ctypes.data, sint.ctypes.data,
                                       s2.ctypes.data), "omr_secret_export")
        return dict(s0=s0, s1=s1, s_int=sint, s2=s2)

    def generate_detection_key(self, seed: int, nthreads: int = 0) -> DetectionKey:
        bsk1 = np.empty(BSK1_SHAPE, np.uint32)
        ksk = np.empty(KSK_SHAPE, np.uint32)
        bsk2 = np.empty(BSK2_SHAPE, np.uint64)
        tk = np.empty(TK_SHAPE, np.uint64)
        _check(lib().omr_keygen_detection_key(self._h, seed, bsk1.reshape(-1), ksk.reshape(-1), bsk2.reshape(-1),
                                              tk.reshape(-1), nthreads), "omr_keygen_detection_key")
        return DetectionKey(bsk1, ksk, bsk2, tk)

    def gen_clues(self, seed: int, first: int, count: int, nthreads: int = 0):
        """Sender::gen_clues for global message indices [first, first+count)."""
        a = np.empty((count, N0), np.uint16)
        b = np.empty((count, CLUE_COUNT), np.uint16)
        _check(lib().omr_gen_clues(self._h, seed, first, count, a.reshape(-1), b.reshape(-1), nthreads),
               "omr_gen_clues")
        return a, b

    # Device generators: same streams, bit-identical results, written to
    # device buffers (ABI layout) of the current HIP device; return when the stream is done.
    def gen_clues_device(self, seed: int, first: int, count: int, d_clue_a: int, d_clue_b: int, stream: int = 0):
        _check(lib().omr_gen_clues_device(self._h, seed, first, count, d_clue_a, d_clue_b, stream or None),
               "omr_gen_clues_device")

    def generate_detection_key_device(self, seed: int, d_bsk1: int, d_ksk: int, d_bsk2: int, d_trace_key: int,
                                      stream: int = 0):
        _check(lib().omr_keygen_detection_key_device(self._h, seed, d_bsk1, d_ksk, d_bsk2, d_trace_key,
                                                     stream or None), "omr_keygen_detection_key_device")


# ---- on-disk container (the reference has no serialization) ----------------
# Little-endian: b"OMRF" | u32 version = 1 | u32 kind | u32 n_arrays | n_arrays x
# {u32 dtype (1 = u16, 2 = u32, 3 = u64), u32 ndim, u64 dims[4]} | arrays in order, each starting
# at a 64-byte aligned offset, C order. Kinds: 1 detection key (bsk1, ksk, bsk2, trace_key in the
# ABI layout of include/omr_gpu.h), 2 clues (clue_a [D][512], clue_b [D][7], first_index [1]),
# 3 NttRlweCiphertexts (u64 [n][2][2048], e.g. a pertinency vector or a digest).
_FILE_MAGIC, _FILE_VERSION = b"OMRF", 1
KIND_DETECTION_KEY, KIND_CLUES, KIND_CIPHERTEXTS = 1, 2, 3
_DT = {np.dtype(np.uint16): 1, np.dtype(np.uint32): 2, np.dtype(np.uint64): 3}
_DT_INV = {v: k for k, v in _DT.items()}


def write_arrays(path: str, kind: int, arrays) -> None:
    arrays = [np.ascontiguousarray(a) for a in arrays]
    head = bytearray(_FILE_MAGIC + np.array([_FILE_VERSION, kind, len(arrays)], "<u4").tobytes())
    for a in arrays:
        if a.dtype not in _DT or a.ndim > 4:
            raise OmrError(f"unsupported array {a.dtype} ndim {a.ndim}")
        dims = list(a.shape) + [0] * (4 - a.ndim)
        head += np.array([_DT[a.dtype], a.ndim], "<u4").tobytes() + np.array(dims, "<u8").tobytes()
    with open(path, "wb") as f:
        f.write(head)
        for a in arrays:
            f.write(b"\0" * (-f.tell() % 64))
            f.write(a.astype(a.dtype.newbyteorder("<"), copy=False).tobytes())


def read_arrays(path: str, kind: int):
    """Arrays of an OMRF file (memory-mapped, read-only) after checking magic, version and kind."""
    with open(path, "rb") as f:
        hdr = f.read(16)
        if len(hdr) < 16 or hdr[:4] != _FILE_MAGIC:
            raise OmrError(f"{path}: not an OMRF file")
        version, k, n = np.frombuffer(hdr[4:16], "<u4")
        if version != _FILE_VERSION or k != kind:
            raise OmrError(f"{path}: version {version} kind {k}, expected {_FILE_VERSION} / {kind}")
        descs = [f.read(40) for _ in range(n)]
        off = f.tell()
    out = []
    for d in descs:
        dt, nd = np.frombuffer(d[:8], "<u4")
        shape = tuple(int(x) for x in np.frombuffer(d[8:], "<u8")[:nd])
        off += -off % 64
        a = np.memmap(path, dtype=_DT_INV[int(dt)].newbyteorder("<"), mode="r", offset=off, shape=shape)
        out.append(a)
        off += a.nbytes
    return out


def save_detection_key(path: str, dk: "DetectionKey") -> None:
    write_arrays(path, KIND_DETECTION_KEY, [dk.bsk1, dk.ksk, dk.bsk2, dk.trace_key])


def load_detection_key(path: str) -> "DetectionKey":
    b1, k, b2, t = read_arrays(path, KIND_DETECTION_KEY)
    return DetectionKey(bsk1=np.array(b1), ksk=np.array(k), bsk2=np.array(b2), trace_key=np.array(t))


def save_clues(path: str, clue_a, clue_b, first: int = 0) -> None:
    write_arrays(path, KIND_CLUES, [np.asarray(clue_a, np.uint16), np.asarray(clue_b, np.uint16),
                                    np.array([first], np.uint64)])


def load_clues(path: str):
    """(clue_a, clue_b, first_index)."""
    a, b, first = read_arrays(path, KIND_CLUES)
    return np.array(a), np.array(b), int(first[0])


def save_ciphertexts(path: str, cts) -> None:
    write_arrays(path, KIND_CIPHERTEXTS, [np.asarray(cts, np.uint64).reshape(-1, 2, N2)])


def load_ciphertexts(path: str) -> np.ndarray:
    return np.array(read_arrays(path, KIND_CIPHERTEXTS)[0])


def fft_twiddles_dd(level: int) -> np.ndarray:
    """The key transform's double-double twiddles [n - 1][4] (re.hi, re.lo, im.hi, im.lo)."""
    n = 512 if level == 1 else 1024
    out = np.zeros(4 * (n - 1), dtype=np.float64)
    _check(lib().omr_fft_twiddles_dd(int(level), out), "omr_fft_twiddles_dd")
    return out.reshape(n - 1, 4)


def detect_kernels() -> dict:
    """{'br1': name, 'ks': name, 'br2': name} of the kernels this build launches."""
    return dict(kv.split("=") for kv in lib().omr_detect_kernels().decode().split())


class Retriever:
    """Retriever (retriever.rs:25-260): client-side digest decoding with the pack's s2 (CPU)."""

    def __init__(self, params: RetrievalParams, secret: "SecretKeyPack"):
        self.params = params
        self._sk = secret

    def decrypt_decode(self, cts) -> np.ndarray:
        """Decoded plaintexts mod 257 of NttRlweCiphertexts u64 [n][2][2048]: u32 [n][2048]."""
        cts = np.ascontiguousarray(cts, dtype=np.uint64).reshape(-1, 2, N2)
        out = np.empty((cts.shape[0], N2), np.uint32)
        _check(lib().omr_decrypt_decode(self._sk._h, cts.reshape(-1), cts.shape[0], out.reshape(-1)),
               "omr_decrypt_decode")
        return out

    def decode_pertinent_indices(self, idx_cts) -> list[int]:
        rp = self.params
        cts = np.ascontiguousarray(idx_cts, dtype=np.uint64).reshape(-1, 2, N2)
        buf = np.zeros(max(1, rp.pertinent_count) * 4 + 64, dtype=np.uintp)
        found = C.c_size_t()
        _check(lib().omr_retrieve_indices(self._sk._h, cts.reshape(-1), cts.shape[0], rp.all_payloads_count,
                                          rp.pertinent_count, buf, buf.size, C.byref(found)),
               "omr_retrieve_indices")
        return [int(v) for v in buf[:min(found.value, buf.size)]]

    def decode_combined_payloads_and_solve(self, pay_cts, weights, indices) -> np.ndarray:
        rp = self.params
        cts = np.ascontiguousarray(pay_cts, dtype=np.uint64).reshape(-1, 2, N2)
        idx = np.ascontiguousarray(sorted(indices), dtype=np.uintp)
        out = np.zeros((len(idx), PAYLOAD_LENGTH), np.uint16)
        _check(lib().omr_retrieve_payloads(self._sk._h, cts.reshape(-1), cts.shape[0], rp.all_payloads_count,
                                           rp.combination_count,
                                           np.ascontiguousarray(weights, dtype=np.uint16).reshape(-1), idx,
                                           len(idx), out.reshape(-1)), "omr_retrieve_payloads")
        return out

    def decode_digest(self, idx_cts, pay_cts, seed: bytes):
        """Retriever::decode_digest: sorted pertinent indices and their payloads (mod 257); the
        weights and the system's rows follow the board's RetrievalParams (retriever.rs:196, :215-239)."""
        indices = self.decode_pertinent_indices(idx_cts)
        weights = payload_weights(seed, self.params)
        return indices, self.decode_combined_payloads_and_solve(pay_cts, weights, indices)


# Contexts still open at interpreter exit are destroyed by an atexit hook, which runs before the
# HIP runtime's own exit-time teardown (a context freed after it faults, e.g. under rocprofv3).
_LIVE_DETECTORS: "weakref.WeakSet[Detector]" = weakref.WeakSet()
_destroy_ctx = None  # omr_ctx_destroy, bound by the first Detector (usable at interpreter shutdown)


def _bind_destroy():
    global _destroy_ctx
    if _destroy_ctx is None:
        _destroy_ctx = lib().omr_ctx_destroy


@atexit.register
def _close_live_detectors():
    for d in list(_LIVE_DETECTORS):
        d.close()


class Detector:
    """Detector (detector.rs:35-453) on one MI355X."""

    def __init__(self, detection_key: DetectionKey, device: int = 0):
        view = _KeyView(detection_key.bsk1.ctypes.data, detection_key.ksk.ctypes.data,
                        detection_key.bsk2.ctypes.data, detection_key.trace_key.ctypes.data)
        for a, shape, dt in ((detection_key.bsk1, BSK1_SHAPE, np.uint32), (detection_key.ksk, KSK_SHAPE, np.uint32),
                             (detection_key.bsk2, BSK2_SHAPE, np.uint64), (detection_key.trace_key, TK_SHAPE, np.uint64)):
            if a.shape != shape or a.dtype != dt or not a.flags.c_contiguous:
                raise OmrError(f"detection key component has shape {a.shape} {a.dtype}, expected {shape} {dt}")
        h = C.c_void_p()
        _check(lib().omr_ctx_create(C.byref(view), device, C.byref(h)), "omr_ctx_create")
        self._h = h
        self.device = device
        _bind_destroy()
        _LIVE_DETECTORS.add(self)

    @classmethod
    def from_device_key(cls, d_bsk1: int, d_ksk: int, d_bsk2: int, d_trace_key: int, device: int = 0):
        """Detector over key components already in the HBM of `device` (device pointers, ABI
        layout), e.g. from SecretKeyPack.generate_detection_key_device."""
        self = cls.__new__(cls)
        view = _KeyView(d_bsk1, d_ksk, d_bsk2, d_trace_key)
        h = C.c_void_p()
        _check(lib().omr_ctx_create(C.byref(view), device, C.byref(h)), "omr_ctx_create")
        self._h = h
        self.device = device
        _bind_destroy()
        _LIVE_DETECTORS.add(self)
        return self

    def close(self):
        if getattr(self, "_h", None):
            (_destroy_ctx or lib().omr_ctx_destroy)(self._h)
            self._h = None

    def __del__(self):
        self.close()

    @property
    def handle(self):
        return self._h

    def set_batch(self, batch: int):
        _check(lib().omr_ctx_set_batch(self._h, batch), "omr_ctx_set_batch")

    def set_encode_chunks(self, max_chunks: int):
        """At most max_chunks partial digests per encode ciphertext (0 = default 4,096)."""
        _check(lib().omr_ctx_set_encode_chunks(self._h, max_chunks), "omr_ctx_set_encode_chunks")

    def set_latency_threshold(self, max_messages: int):
        """Chunks of at most max_messages messages use the latency kernels (0: never)."""
        _check(lib().omr_ctx_set_latency_threshold(self._h, max_messages), "omr_ctx_set_latency_threshold")

    def set_exact_level1(self, enable: bool = True):
        """Level 1 on the exact modular NTT for every launch (omr_ctx_set_exact_level1: the
        reference's arithmetic, bit-identical outputs, slower); False restores the FFT kernels."""
        _check(lib().omr_ctx_set_exact_level1(self._h, 1 if enable else 0), "omr_ctx_set_exact_level1")

    # detect (detector.rs:135) — one clue set -> NttRlweCiphertext [2][2048]
    def detect(self, clue_a, clue_b) -> np.ndarray:
        """One message (omr_detect): thread-safe; concurrent callers are coalesced into batched
        launches (ctypes releases the GIL during the call)."""
        a = np.ascontiguousarray(clue_a, dtype=np.uint16).reshape(N0)
        b = np.ascontiguousarray(clue_b, dtype=np.uint16).reshape(CLUE_COUNT)
        out = np.empty((2, N2), np.uint64)
        _check(lib().omr_detect(self._h, a, b, out.reshape(-1)), "omr_detect")
        return out

    def set_coalescing(self, max_messages: int = 0, window_us: int = 0):
        _check(lib().omr_ctx_set_coalescing(self._h, int(max_messages), int(window_us)), "omr_ctx_set_coalescing")

    def coalescing_stats(self) -> tuple:
        calls, launches = C.c_size_t(), C.c_size_t()
        _check(lib().omr_ctx_coalescing_stats(self._h, C.byref(calls), C.byref(launches)), "omr_ctx_coalescing_stats")
        return calls.value, launches.value

    def detect_batch(self, clue_a, clue_b) -> np.ndarray:
        clue_a = np.ascontiguousarray(clue_a, dtype=np.uint16)
        clue_b = np.ascontiguousarray(clue_b, dtype=np.uint16)
        D = clue_a.shape[0]
        if clue_a.shape != (D, N0) or clue_b.shape != (D, CLUE_COUNT):
            raise OmrError("clues must be u16 [D][512] and [D][7]")
        out = np.empty((D, 2, N2), np.uint64)
        _check(lib().omr_detect_batch(self._h, clue_a.reshape(-1), clue_b.reshape(-1), D, out.reshape(-1)),
               "omr_detect_batch")
        return out

    def detect_batch_device(self, d_clue_a: int, d_clue_b: int, D: int, d_out: int, stream: int = 0):
        _check(lib().omr_detect_batch_device(self._h, d_clue_a, d_clue_b, D, d_out, stream or None),
               "omr_detect_batch_device")

    def check(self, stream: int = 0):
        """omr_ctx_check: sync `stream` (0: the whole device) and raise if an earlier call's device
        work failed."""
        _check(lib().omr_ctx_check(self._h, stream or None), "omr_ctx_check")

    def set_rounding_guard(self, enable: bool = True):
        """Run the guarded FFT kernel variants (same output) that record the rounding margin."""
        _check(lib().omr_ctx_set_rounding_guard(self._h, int(bool(enable))), "omr_ctx_set_rounding_guard")

    def rounding_margin(self, reset: bool = False) -> dict:
        """{"observed": [level1, level2] largest |y - rint(y)| of the guarded runs so far,
        "apriori": [E1, E2] proven bounds on |computed - exact|, "kappa": key-spectrum maxima}."""
        obs, apr, kap = (C.c_double * 2)(), (C.c_double * 2)(), (C.c_double * 2)()
        _check(lib().omr_ctx_rounding_margin(self._h, obs, apr, kap, int(bool(reset))), "omr_ctx_rounding_margin")
        return {"observed": list(obs), "apriori": list(apr), "kappa": list(kap)}

    def exactness(self) -> dict:
        """The exactness contract (omr_ctx_exactness): {"guarded": [l1, l2] guarded on every launch
        (automatically when the key's a priori bound E >= 0.5), "breaches": [l1, l2] launches whose
        margin reached 1 - E (each such launch re-run on the exact NTT)}."""
        g, b = (C.c_int * 2)(), (C.c_uint64 * 2)()
        _check(lib().omr_ctx_exactness(self._h, g, b), "omr_ctx_exactness")
        return {"guarded": [bool(v) for v in g], "breaches": list(b)}

    def key_spectrum(self, level: int, first: int, count: int) -> np.ndarray:
        """Stored key-spectrum values [count] complex (omr_ctx_key_spectrum)."""
        out = np.zeros(2 * count, dtype=np.float64)
        _check(lib().omr_ctx_key_spectrum(self._h, int(level), int(first), int(count), out), "omr_ctx_key_spectrum")
        return out.view(np.complex128)

    def enable_timing(self, mode: int = 1):
        """0 off; 1 stage events around the production kernels; 2 the reference's split (the
        trace as its own launch: the throughput path's production form since round 5)."""
        _check(lib().omr_ctx_enable_timing(self._h, int(mode)), "omr_ctx_enable_timing")

    def last_timing(self) -> dict:
        t = _Timing()
        _check(lib().omr_last_timing(self._h, C.byref(t)), "omr_last_timing")
        return {n: getattr(t, n) for n, _ in _Timing._fields_}

    # detect_with_time_info (detector.rs:169-221): DetectTimeInfo of one batch (device time),
    # detect + timing in one locked call
    def detect_with_time_info(self, clue_a, clue_b):
        clue_a = np.ascontiguousarray(clue_a, dtype=np.uint16)
        clue_b = np.ascontiguousarray(clue_b, dtype=np.uint16)
        D = clue_a.shape[0]
        if clue_a.shape != (D, N0) or clue_b.shape != (D, CLUE_COUNT):
            raise OmrError("clues must be u16 [D][512] and [D][7]")
        out = np.empty((D, 2, N2), np.uint64)
        t = _Timing()
        _check(lib().omr_detect_with_time_info(self._h, clue_a.reshape(-1), clue_b.reshape(-1), D, out.reshape(-1),
                                               C.byref(t)), "omr_detect_with_time_info")
        return out, {n: getattr(t, n) for n, _ in _Timing._fields_}

    # encode_pertinent_indices (detector.rs:223-339)
    def encode_pertinent_indices(self, rp: RetrievalParams, pertinency_vector, seed: int, ct: int = 0,
                                 global_offset: int = 0) -> np.ndarray:
        pv = np.ascontiguousarray(pertinency_vector, dtype=np.uint64)
        D = pv.shape[0]
        out = np.empty((2, N2), np.uint64)
        _check(lib().omr_encode_indices(self._h, pv.reshape(-1), D, global_offset, rp.all_payloads_count, seed, ct,
                                        out.reshape(-1)), "omr_encode_indices")
        return out

    # encode_pertinent_payloads (detector.rs:341-453)
    def encode_pertinent_payloads(self, pertinency_vector, payloads, weights, rp: RetrievalParams,
                                  global_offset: int = 0) -> np.ndarray:
        pv = np.ascontiguousarray(pertinency_vector, dtype=np.uint64)
        pay = np.ascontiguousarray(payloads, dtype=np.uint16)
        w = np.ascontiguousarray(weights, dtype=np.uint16)
        D = pv.shape[0]
        n_ct, per = rp.cmb_cipher_count, rp.cmb_count_per_cipher
        out = np.empty((n_ct, 2, N2), np.uint64)
        _check(lib().omr_encode_payloads(self._h, pv.reshape(-1), pay.reshape(-1), D, global_offset,
                                         rp.all_payloads_count, w, n_ct, per, out.reshape(-1)), "omr_encode_payloads")
        return out

    # device-pointer variants (chaining on the caller's HIP stream; pointers are raw addresses)
    def encode_indices_device(self, d_pv: int, D: int, global_offset: int, all_payloads_count: int, seed: int,
                              first_ct: int, n_ct: int, d_out: int, stream: int = 0) -> None:
        _check(lib().omr_encode_indices_device(self._h, d_pv, D, global_offset, all_payloads_count, seed, first_ct,
                                               n_ct, d_out, stream or None), "omr_encode_indices_device")

    def encode_payloads_device(self, d_pv: int, d_payloads: int, D: int, global_offset: int,
                               all_payloads_count: int, d_weights: int, n_ct: int, per_ct: int, d_out: int,
                               stream: int = 0) -> None:
        _check(lib().omr_encode_payloads_device(self._h, d_pv, d_payloads, D, global_offset, all_payloads_count,
                                                d_weights, n_ct, per_ct, d_out, stream or None),
               "omr_encode_payloads_device")

    # ---- stage entry points (benches/two_level_bs.rs) ----
    def first_level(self, clue_a, clue_b) -> np.ndarray:
        clue_a = np.ascontiguousarray(clue_a, dtype=np.uint16).reshape(-1, N0)
        clue_b = np.ascontiguousarray(clue_b, dtype=np.uint16).reshape(-1, CLUE_COUNT)
        out = np.empty((clue_a.shape[0], NI + 1), np.uint32)
        _check(lib().omr_first_level(self._h, clue_a.reshape(-1), clue_b.reshape(-1), clue_a.shape[0],
                                     out.reshape(-1)), "omr_first_level")
        return out

    def blind_rotate_level1(self, lwe_a, lwe_b) -> np.ndarray:
        lwe_a = np.ascontiguousarray(lwe_a, dtype=np.uint16).reshape(-1, N0)
        lwe_b = np.ascontiguousarray(lwe_b, dtype=np.uint16).reshape(-1)
        out = np.empty((lwe_a.shape[0], 2, N1), np.uint64)
        _check(lib().omr_blind_rotate_level1(self._h, lwe_a.reshape(-1), lwe_b, lwe_a.shape[0], out.reshape(-1)),
               "omr_blind_rotate_level1")
        return out

    def fft1_mul(self, a, k) -> np.ndarray:
        """a * k mod (X^1024 + 1, q1) through the level-1 FFT path (a digit-sized)."""
        a = np.ascontiguousarray(a, dtype=np.uint32).reshape(-1, N1)
        k = np.ascontiguousarray(k, dtype=np.uint32).reshape(-1, N1)
        out = np.empty(a.shape, np.uint64)
        _check(lib().omr_fft1_mul(self._h, a.reshape(-1), k.reshape(-1), a.shape[0], out.reshape(-1)),
               "omr_fft1_mul")
        return out

    def second_level(self, lwe_int) -> np.ndarray:
        lwe = np.ascontiguousarray(lwe_int, dtype=np.uint32).reshape(-1, NI + 1)
        out = np.empty((lwe.shape[0], 2, N2), np.uint64)
        _check(lib().omr_second_level(self._h, lwe.reshape(-1), lwe.shape[0], out.reshape(-1)), "omr_second_level")
        return out

    def blind_rotate_level2(self, lwe_int) -> np.ndarray:
        lwe = np.ascontiguousarray(lwe_int, dtype=np.uint32).reshape(-1, NI + 1)
        out = np.empty((lwe.shape[0], 2, N2), np.uint64)
        _check(lib().omr_blind_rotate_level2(self._h, lwe.reshape(-1), lwe.shape[0], out.reshape(-1)),
               "omr_blind_rotate_level2")
        return out


def ntt(level: int, polys, inverse: bool = False, device: int = 0) -> np.ndarray:
    p = np.array(polys, dtype=np.uint64, copy=True)
    n = (1024 if level == 1 else 2048)
    p2 = p.reshape(-1, n)
    flat = np.ascontiguousarray(p2).reshape(-1)
    _check(lib().omr_ntt(level, int(inverse), flat, p2.shape[0], device), "omr_ntt")
    return flat.reshape(p.shape)


class KeyGen:
    """KeyGen::generate_secret_key (key_gen/mod.rs:21-27)."""

    @staticmethod
    def generate_secret_key(seed: int) -> SecretKeyPack:
        return SecretKeyPack(seed)
