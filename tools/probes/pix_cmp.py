import numpy as np, sys
NC = 512
a = np.fromfile(sys.argv[1], np.uint8); b = np.fromfile(sys.argv[2], np.uint8)
da, db = a[:NC * 4096].reshape(NC, 4096), b[:NC * 4096].reshape(NC, 4096)
ra, rb = a[NC * 4096:].view(np.uint32).reshape(NC, 4), b[NC * 4096:].view(np.uint32).reshape(NC, 4)
bad = [i for i in range(NC) if (da[i] != db[i]).any() or (ra[i] != rb[i]).any()]
print("mismatching cases", len(bad))
ws = [4, 8, 16, 32, 64, 2]
for i in bad[:20]:
    k = i % 8; w = ws[(i // 8) % 6]; h = ws[(i // 48) % 5]
    print(i, "kind", k, "w", w, "h", h, "res", ra[i], rb[i], "first px diff", np.flatnonzero(da[i] != db[i])[:5])
