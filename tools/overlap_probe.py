"""Probe (round 6): does running level 1 of one chunk beside level 2 of another raise throughput?

Two contexts on two HIP streams share the GPU: context A detects half of the D messages in chunks
of D/4, context B the other half, its first chunk D/8 long so that its level 1 runs while A is in
level 2 (the rotations then share CUs: br1f 76 KB + br2f 80 KB of LDS fit one CU). Against one
context detecting D in one launch per stage, and one context detecting D in chunks of D/4 (the
chunking's own cost). Outputs are checked against the single-launch run.
    python tools/overlap_probe.py [D]
"""
import sys
import time

import numpy as np
import torch

sys.path.insert(0, "tfhe-omr_amd")
import omr_amd as A  # noqa: E402

D = int(sys.argv[1]) if len(sys.argv) > 1 else 65536
dev = torch.device("cuda:0")
torch.cuda.set_device(dev)
pack = A.SecretKeyPack(42)
cur = torch.cuda.current_stream(dev).cuda_stream
kb = [torch.empty(int(np.prod(s)), dtype=t, device=dev)
      for s, t in ((A.BSK1_SHAPE, torch.int32), (A.KSK_SHAPE, torch.int32),
                   (A.BSK2_SHAPE, torch.int64), (A.TK_SHAPE, torch.int64))]
pack.generate_detection_key_device(7, *[b.data_ptr() for b in kb], stream=cur)
da = A.Detector.from_device_key(*[b.data_ptr() for b in kb])
db = A.Detector.from_device_key(*[b.data_ptr() for b in kb])
ca = torch.empty((D, A.N0), dtype=torch.int16, device=dev)
cb = torch.empty((D, A.CLUE_COUNT), dtype=torch.int16, device=dev)
pack.gen_clues_device(1000, 0, D, ca.data_ptr(), cb.data_ptr(), stream=cur)
ref = torch.empty((D, 2, 2048), dtype=torch.int64, device=dev)
out = torch.empty_like(ref)
sa, sb = torch.cuda.Stream(dev), torch.cuda.Stream(dev)
torch.cuda.synchronize(dev)


def run(det, lo, hi, stream, o):
    det.detect_batch_device(ca[lo:].data_ptr(), cb[lo:].data_ptr(), hi - lo, o[lo:].data_ptr(), stream.cuda_stream)


def timed(fn):
    torch.cuda.synchronize(dev)
    t = time.perf_counter()
    fn()
    torch.cuda.synchronize(dev)
    return (time.perf_counter() - t) * 1e3


def single():
    da.set_batch(D)
    run(da, 0, D, sa, ref)


def chunked():
    da.set_batch(D // 4)
    run(da, 0, D, sa, out)


def overlap():
    da.set_batch(D // 4)
    db.set_batch(D // 4)
    h, e = D // 2, D // 8
    run(da, 0, h, sa, out)
    run(db, h, h + e, sb, out)
    run(db, h + e, D, sb, out)


single()  # warm-up
for rep in range(2):
    ms = timed(single)
    print(f"single launch per stage: {ms:.0f} ms  {D / ms * 1e3:.0f} msg/s", flush=True)
    ms = timed(chunked)
    ok = torch.equal(out, ref)
    print(f"one context, chunks of D/4: {ms:.0f} ms  {D / ms * 1e3:.0f} msg/s  identical={ok}", flush=True)
    out.zero_()
    ms = timed(overlap)
    ok = torch.equal(out, ref)
    print(f"two contexts, two streams, offset chunks: {ms:.0f} ms  {D / ms * 1e3:.0f} msg/s  identical={ok}",
          flush=True)
da.close()
db.close()
