"""Summarise a per-tile timestamp trace written by scripts/ubench_rl.bin -DTRACE:
u64[tiles][8] s_memrealtime (100 MHz): 0 ticket, 1 all waves scanned, 2 map
published, 3 look-back resolved, 4 wave 0 emitted (flrl_rl.hip FLRL_RL_TRACE)."""
import sys

import numpy as np

raw = np.fromfile(sys.argv[1], dtype=np.uint64).reshape(-1, 8)
t = raw[:, :5].astype(np.int64)
spins, rounds = raw[:, 5].astype(np.int64), raw[:, 6].astype(np.int64)
t0 = t[t > 0].min()
t = (t - t0) * 10 / 1000.0  # us
start, scanned, pub, lb, end = t[:, 0], t[:, 1], t[:, 2], t[:, 3], t[:, 4]
print(f"tiles {len(t)}  span {end.max() - start.min():.1f} us")


def pct(x, name):
    print(f"{name:34s} p10 {np.percentile(x, 10):7.2f}  p50 {np.percentile(x, 50):7.2f}  "
          f"p90 {np.percentile(x, 90):7.2f}  mean {x.mean():7.2f}")


pct(scanned - start, "start -> all waves scanned")
pct(pub - scanned, "scanned -> map published")
pct(lb - pub, "published -> look-back resolved")
pct(end - lb, "resolved -> stores issued")
pct(pub[1:] - pub[:-1], "pub[t] - pub[t-1]")
print("fraction of tiles whose predecessor published later:", round(float((pub[:-1] > pub[1:]).mean()), 3))
pct(lb[1:] - lb[:-1], "lb[t] - lb[t-1]")
i = len(t) // 2
print("look-back spins: mean", round(float(spins.mean()), 2), "p90", int(np.percentile(spins, 90)),
      "| windows: mean", round(float(rounds.mean()), 2), "p90", int(np.percentile(rounds, 90)), "max", int(rounds.max()))
busy = np.zeros(int(end.max()) + 2)
for a, b in zip(start, end):  # tiles in flight per us
    busy[int(a):int(b) + 1] += 1
print("tiles in flight: mean", round(float(busy[busy > 0].mean()), 1), "max", int(busy.max()))
w = lb - pub
print("look-back wait share of tile time:", round(float(w.sum() / (end - start).sum()), 3))
for k in range(i, i + 10):
    print(k, *(round(float(v), 2) for v in t[k]))
# occupancy over the launch: tiles in flight per 10 us bin, and the share of
# slot-time lost to the ramp-up and the tail (against the peak occupancy)
peak = int(np.percentile(busy[busy > 0], 90))
bins = [int(busy[k:k + 10].mean()) for k in range(0, len(busy), 10)]
print("in flight per 10 us:", bins)
span = float(end.max() - start.min())
print("slot-time lost vs p90 occupancy", peak, ":", round(float(np.clip(peak - busy[:int(span)], 0, None).sum() / (peak * span)), 3))
last = np.sort(start)[-peak:]
print("last", peak, "tiles: started", round(float(last.min()), 1), "..", round(float(last.max()), 1), "us; kernel end", round(float(end.max()), 1))
