"""Shared fixtures: the product's Python host mirror (tfhe-omr_amd/omr_amd.py)."""
import functools
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tfhe-omr_amd"))
import omr_amd  # noqa: E402

KEY_SEED, SK_SEED, SK2_SEED = 7, 42, 4242


@functools.lru_cache(maxsize=1)
def keys():
    """Pack A (the detector's recipient), pack B (non-pertinent senders), A's detection key."""
    a = omr_amd.SecretKeyPack(SK_SEED)
    b = omr_amd.SecretKeyPack(SK2_SEED)
    dk = a.generate_detection_key(KEY_SEED)
    return a, b, dk


def mixed_clues(pertinent_mask, seed=1000, first=0):
    """Clues for global indices first..first+D: from pack A where pertinent, else pack B."""
    import numpy as np
    a, b, _ = keys()
    D = len(pertinent_mask)
    ca, cb = a.gen_clues(seed, first, D)
    na, nb = b.gen_clues(seed + 1, first, D)
    m = np.asarray(pertinent_mask, dtype=bool)
    ca[~m] = na[~m]
    cb[~m] = nb[~m]
    return ca, cb
