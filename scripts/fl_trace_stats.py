"""Summarise the FL encode per-tile trace of scripts/ubench_fl.bin -DTRACE:
u64[tiles][4] s_memrealtime (100 MHz): 0 tile start (ticket), 1 widths done /
aggregate published, 2 look-back resolved, 3 stores issued (flrl_fl.hip
FLRL_FL_TRACE). Prints per-phase percentiles, the tile period per workgroup
and the grid's start-up and tail."""
import sys

import numpy as np

raw = np.fromfile(sys.argv[1], dtype=np.uint64).reshape(-1, 4).astype(np.int64)
ok = (raw > 0).all(axis=1)
t = raw[ok]
t0 = t.min()
t = (t - t0) * 10 / 1000.0  # us
start, pub, lb, end = t[:, 0], t[:, 1], t[:, 2], t[:, 3]
print(f"tiles {len(t)} (of {len(raw)})  span {end.max():.1f} us  first stores issued {end.min():.1f} us")


def pct(x, name):
    print(f"{name:34s} p10 {np.percentile(x, 10):7.2f}  p50 {np.percentile(x, 50):7.2f}  "
          f"p90 {np.percentile(x, 90):7.2f}  mean {x.mean():7.2f}")


pct(pub - start, "start -> widths/published")
pct(lb - pub, "published -> resolved")
pct(end - lb, "resolved -> stores issued")
pct(end - start, "tile life")
order = np.argsort(start)
gaps = np.diff(start[order])
print("tile starts per us (steady state):", round(len(t) / (start.max() - start.min()), 2))
tail = end.max() - np.percentile(end, 99)
print(f"last 1 % of stores issued over {tail:.1f} us; start-up: 99 % of first-round tiles started by "
      f"{np.percentile(start[:256], 99):.1f} us")
# launch overhead against the steady state: tiles completed per us over the
# middle 80 % of completions, the span that rate would need for all tiles,
# and where the rest goes (ramp: first completion; tail: last 256 completions)
done = np.sort(end)
k0, k1 = int(0.1 * len(done)), int(0.9 * len(done))
rate = (k1 - k0) / (done[k1] - done[k0])
print(f"steady completions {rate:.2f} tiles/us -> ideal span {len(done) / rate:.1f} us vs {done[-1]:.1f} us; "
      f"first completion {done[0]:.1f} us, 256th {done[min(255, len(done) - 1)]:.1f} us, "
      f"last 256 completions over {done[-1] - done[max(0, len(done) - 256)]:.1f} us "
      f"(steady: {256 / rate:.1f} us)")
