import sys, numpy as np
a = np.fromfile(sys.argv[1], dtype=np.uint64).reshape(-1, 16)
na = int(sys.argv[2])
a = a[:na]
ok = (a[:, 0] > 0) & (a[:, 2] < 0xfffff) & (a[:, 2] >= 128)
a = a[ok].astype(np.int64)
ev = a[:, 2]
t = lambda c: (a[:, c] - a[:, 0]) * 10 / 1000.0
cols = {"setup(a)": 4, "staging": 5, "pairs+prefix": 6, "circle3 tasks": 7, "circle4": 8, "flags/end": 1}
prev = np.zeros(len(a))
print("n staged items", len(a), "events p50", np.median(ev))
for name, c in cols.items():
    cur = t(c)
    print(f"{name:14s} phase p50 {np.median(cur - prev):5.2f} us  p90 {np.percentile(cur - prev, 90):5.2f}  (cum p50 {np.median(cur):5.2f})")
    prev = cur
