"""Expand the structured-key descriptions stored in tests/golden/structured_detect.npz into the
canonical coefficient-domain key arrays of include/omr_gpu.h (test infrastructure)."""
from __future__ import annotations

import functools
import os

import numpy as np

import omr_model as M

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


@functools.lru_cache(maxsize=1)
def load():
    z = np.load(os.path.join(GOLDEN, "structured_detect.npz"))
    s1 = [tuple(int(v) for v in r) for r in z["s1"]]
    s2 = [tuple(int(v) for v in r) for r in z["s2"]]

    def ggsw(alpha, noise, bits, which):
        return [M.StructuredGGSW(which, int(b), [tuple(int(v) for v in r) for r in a],
                                 [tuple(int(v) for v in r) for r in e]) for a, e, b in zip(alpha, noise, bits)]

    bsk1 = ggsw(z["bsk1_alpha"], z["bsk1_noise"], z["s0"], 1)
    bsk2 = ggsw(z["bsk2_alpha"], z["bsk2_noise"], z["sint"], 2)
    tk = []
    for k in range(M.TRACE_STEPS):
        g = (M.N2 >> k) + 1
        rows = [(tuple(int(v) for v in z["tk_alpha"][k, j]), tuple(int(v) for v in z["tk_noise"][k, j]))
                for j in range(M.DT)]
        tk.append((g, M.sparse_auto(s2, g, M.N2), rows))
    keys = dict(
        bsk1=M.dense_bsk(1, bsk1, s1).astype(np.uint32),
        bsk2=M.dense_bsk(2, bsk2, s2),
        ksk=M.ksk_dense(int(z["ksk_seed"])).astype(np.uint32).reshape(M.N1, M.KS_DIGITS, M.NI + 1),
        tk=M.dense_trace_key(tk, s2),
    )
    expect = {k: z[k] for k in ("clue_a", "clue_b", "br1_clue0", "lwe_int", "br2", "detect")}
    return keys, expect
