"""Where the RL encode's per-tile scan-time spread comes from.

Reads a per-tile trace of scripts/ubench_rl_TRACE.bin (u64[tiles][8]: 0 start,
1 all waves scanned, 2 published, 3 resolved, 4 emitted, 5 spins, 6 windows,
7 XCC id << 32 | HW_ID) and optionally the input it encoded (INPUT_OUT), and
correlates each tile's scan time (start -> scanned) with
  - data: the tile's natural heads (runs starting in it),
  - placement: its XCC, its CU (XCC, SE, SH, CU), its SIMD/wave slot,
  - time: its start time (launch ramp vs steady state, tail).
Usage: python3 scripts/trace_where.py trace.bin [input.bin]"""
import sys

import numpy as np

raw = np.fromfile(sys.argv[1], dtype=np.uint64).reshape(-1, 8)
T = raw.shape[0]
t = raw[:, :5].astype(np.int64)
t0 = t[t > 0].min()
t = (t - t0) * 10 / 1000.0  # us (s_memrealtime: 100 MHz)
start, scanned, pub, lb, end = (t[:, i] for i in range(5))
scan = scanned - start
where = raw[:, 7]
xcc = (where >> np.uint64(32)).astype(np.int64) & 0xF
hw = (where & np.uint64(0xFFFFFFFF)).astype(np.int64)
wave_id, simd, cu, sh, se = hw & 0xF, (hw >> 4) & 3, (hw >> 8) & 0xF, (hw >> 12) & 1, (hw >> 13) & 7
cu_key = ((xcc * 8 + se) * 2 + sh) * 16 + cu
print(f"tiles {T}  span {end.max() - start.min():.1f} us  scan p10/p50/p90 "
      f"{np.percentile(scan, 10):.2f} / {np.percentile(scan, 50):.2f} / {np.percentile(scan, 90):.2f} us")
print(f"distinct XCCs {len(set(xcc))}, CUs {len(set(cu_key))}")


def explained(groups, name):
    """share of the scan-time variance explained by the group means"""
    tot = scan.var()
    means = {g: scan[groups == g].mean() for g in set(groups)}
    fit = np.array([means[g] for g in groups])
    print(f"{name:28s} groups {len(means):5d}  R^2 {1 - ((scan - fit) ** 2).mean() / tot:.3f}  "
          f"group-mean range {min(means.values()):.2f} .. {max(means.values()):.2f} us")
    return means


mx = explained(xcc, "XCC")
for g in sorted(mx):
    print(f"   XCC {g}: tiles {int((xcc == g).sum())}  mean scan {mx[g]:.2f} us")
explained(cu_key, "CU")
explained(simd + 4 * cu_key, "CU x SIMD")
# time: 10 us bins of start time
explained((start // 10).astype(np.int64), "start time (10 us bins)")
explained(np.arange(T) % 8, "tile mod 8")
if len(sys.argv) > 2:
    x = np.fromfile(sys.argv[2], dtype=np.uint8)
    TB = (x.size + T - 1) // T
    TB = 1 << int(np.ceil(np.log2(TB)))  # tile bytes (128 KiB)
    heads = np.concatenate([[1], (x[1:] != x[:-1]).astype(np.uint8)])
    nh = np.add.reduceat(heads, np.arange(0, x.size, TB))[:T].astype(np.float64)
    c = np.corrcoef(nh, scan)[0, 1]
    print(f"natural heads per tile: mean {nh.mean():.0f} sd {nh.std():.1f}  corr(heads, scan) {c:.3f}  R^2 {c * c:.3f}")
# the look-back waits on the slowest predecessor: how often is the blocking
# predecessor (the latest-published of the 64 before) on another XCC?
late = np.array([k - 64 + int(np.argmax(pub[max(0, k - 64):k])) if k else 0 for k in range(T)])
late[:1] = 0
print("tile's latest-published predecessor on the same XCC:", round(float((xcc[late] == xcc).mean()), 3))
print("mean wait published -> resolved:", round(float((lb - pub).mean()), 2), "us")
