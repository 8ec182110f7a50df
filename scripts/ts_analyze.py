import sys, numpy as np
a = np.fromfile(sys.argv[1], dtype=np.uint64).reshape(-1, 16)[:, :4]
nb = int(sys.argv[2])
used = np.nonzero(a[:, 0])[0]
a = a[: used.max() + 1]
t0 = a[a[:, 0] > 0, 0].min()
st = (a[:, 0].astype(np.int64) - int(t0)) * 10 / 1000.0  # us (100 MHz)
en = (a[:, 1].astype(np.int64) - int(t0)) * 10 / 1000.0
d = en - st
print(f"WGs={len(a)} span={en.max():.1f}us build={nb}")
na = int(sys.argv[3]) if len(sys.argv) > 3 else 0
b, r = (slice(na, len(a)), slice(0, na)) if na else (slice(0, nb), slice(nb, len(a)))
for name, sl in (("build", b), ("arc", r)):
    x = d[sl]; s0 = st[sl]
    print(f"{name:5s} dur p10/50/90/max {np.percentile(x,10):.1f} {np.median(x):.1f} {np.percentile(x,90):.1f} {x.max():.1f}  start p50/90/max {np.median(s0):.1f} {np.percentile(s0,90):.1f} {s0.max():.1f}  end max {en[sl].max():.1f}")
xcc = a[:, 3] & 0xf
print("WGs per XCC:", np.bincount(xcc.astype(np.int64), minlength=8))
arc_d = d[r]; big = np.argsort(-arc_d)[:8]; off = r.start
print("slowest arc WGs (idx, start, dur):", [(int(i), round(float(st[off + i]), 1), round(float(arc_d[i]), 1)) for i in big])
hist = np.histogram(st, bins=10)
print("start histogram:", hist[0], np.round(hist[1], 1))
ev = a[:, 2].astype(np.int64)
if na:
    e = ev[:na]; dd = d[:na]; m = e < 0xfffff
    print("arc items: events vs duration (deciles of events)")
    for lo, hi in [(0, 128), (128, 512), (512, 1024), (1024, 1900), (1900, 2049)]:
        sel = m & (e >= lo) & (e < hi)
        if sel.any(): print(f"  events [{lo},{hi}): n={sel.sum()} dur p50={np.median(dd[sel]):.1f} max={dd[sel].max():.1f}")
    print("slowest:", [(int(i), int(e[i]), round(float(dd[i]), 1)) for i in np.argsort(-dd)[:6]])
