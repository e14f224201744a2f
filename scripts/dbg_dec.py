"""Decode probe (GPU box): errors, round trip, and the tagged tile offsets of
the fused FL decode against the widths."""
import sys, os
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "fl-rl-compression-mpi_amd"))
import numpy as np
import torch
import flrl
from flrl.device import FLDevice, gen
for n in [int(a) for a in sys.argv[1:]]:
    x = gen("u8", n, 42)
    d = FLDevice(n)
    d.encode(x)
    v = d.values_size()
    e0 = d.error()
    out = d.decode(v)
    torch.cuda.synchronize()
    ok = bool(torch.equal(out, x[:n]))
    print(n, "enc err", e0, "dec err", d.error(), "ok", ok, flush=True)
    if not ok:
        bad = (out != x[:n]).nonzero()
        print("  first bad byte", int(bad[0]), "count", bad.numel(), flush=True)
    ntiles = -(-n // 65536)
    tb = max(1, min(64, -(-ntiles // 512)))
    nb = -(-ntiles // tb)
    off = 16 + nb * 128
    raw = d.scratch[off:off + 8 * (ntiles + 1)].cpu().numpy().view(np.uint64)
    w = np.clip(d.bits[:d.frames].cpu().numpy().astype(np.int64), 1, 8)
    ref = np.concatenate([[0], np.cumsum([w[t * 512:(t + 1) * 512].sum() for t in range(ntiles)])])
    got = (raw & np.uint64((1 << 63) - 1)).astype(np.int64)
    tags = (raw >> np.uint64(63)).astype(np.int64)
    if not (np.array_equal(got, ref) and tags.all()):
        print("  tile_base mismatch:", [(t, int(got[t]), int(ref[t]), int(tags[t])) for t in range(ntiles + 1)
                                       if got[t] != ref[t] or not tags[t]][:10], flush=True)
