"""Independent numpy restatement of the synthetic generators (DESIGN.md §5,
SURVEY.md §8(d) table: C3/C4 stripe CSR, C5 R-MAT) and of the input
vectors the golden vectors use.  Test infrastructure: it pins the product's
C++ generator (host/Synthetic.cpp) and feeds make_vectors.py."""
import numpy as np

GOLDEN = 0x9E3779B97F4A7C15
M1 = 0xBF58476D1CE4E5B9
M2 = 0x94D049BB133111EB


def splitmix64_at(seed: int, i) -> np.ndarray:
    """i-th output of splitmix64 seeded with `seed` (Vigna), vectorised over i."""
    i = np.asarray(i, dtype=np.uint64)
    with np.errstate(over="ignore"):
        z = np.uint64(seed) + (i + np.uint64(1)) * np.uint64(GOLDEN)
        z = (z ^ (z >> np.uint64(30))) * np.uint64(M1)
        z = (z ^ (z >> np.uint64(27))) * np.uint64(M2)
    return z ^ (z >> np.uint64(31))


def uniform11(z: np.ndarray) -> np.ndarray:
    """(z >> 11) * 2^-52 - 1: exact doubles in [-1, 1)."""
    return (z >> np.uint64(11)).astype(np.float64) * 2.0 ** -52 - 1.0


def vector_f64(n: int, seed: int) -> np.ndarray:
    return uniform11(splitmix64_at(seed, np.arange(n, dtype=np.uint64)))


def vector_u64(n: int, seed: int) -> np.ndarray:
    return splitmix64_at(seed, np.arange(n, dtype=np.uint64))


def stripe_csr(row0: int, nrows: int, cols: int, k: int = 32, seed_col: int = 1, seed_val: int = 2):
    """Row r has k columns, one per stripe [j*cols/k, (j+1)*cols/k):
    col_j = lo_j + splitmix64_at(seed_col, r*k+j) mod width_j, value
    uniform11(splitmix64_at(seed_val, r*k+j))."""
    lo = (np.arange(k + 1, dtype=np.uint64) * np.uint64(cols)) // np.uint64(k)
    width = (lo[1:] - lo[:-1])
    g = (np.uint64(row0) + np.arange(nrows, dtype=np.uint64))[:, None] * np.uint64(k) + np.arange(k, dtype=np.uint64)
    colind = (lo[:-1] + splitmix64_at(seed_col, g) % width).astype(np.uint32).ravel()
    vals = uniform11(splitmix64_at(seed_val, g)).ravel()
    rowptr = (np.arange(nrows + 1, dtype=np.uint64) * np.uint64(k)).astype(np.uint32)
    return rowptr, colind, vals


def rmat_csr(scale: int, edge_factor: int = 16, seed: int = 4, a=0.57, b=0.19, c=0.19):
    """Graph500 R-MAT: edge i picks a quadrant per level from
    u = (splitmix64_at(seed, i*scale+lvl) >> 11) * 2^-53; value
    uniform11(splitmix64_at(seed+1, i)); edges sorted by (row, col), stable,
    duplicates summed in edge order."""
    n = 1 << scale
    m = n * edge_factor
    i = np.arange(m, dtype=np.uint64)
    r = np.zeros(m, dtype=np.uint64)
    cc = np.zeros(m, dtype=np.uint64)
    for lvl in range(scale):
        u = (splitmix64_at(seed, i * np.uint64(scale) + np.uint64(lvl)) >> np.uint64(11)).astype(np.float64) * 2.0 ** -53
        bit = np.uint64(1 << (scale - 1 - lvl))
        q_col = (u >= a) & (u < a + b)
        q_row = (u >= a + b) & (u < a + b + c)
        q_both = u >= a + b + c
        cc |= np.where(q_col | q_both, bit, np.uint64(0))
        r |= np.where(q_row | q_both, bit, np.uint64(0))
    v = uniform11(splitmix64_at(seed + 1, i))
    key = (r << np.uint64(32)) | cc
    order = np.argsort(key, kind="stable")
    key, v = key[order], v[order]
    first = np.ones(m, dtype=bool)
    first[1:] = key[1:] != key[:-1]
    starts = np.nonzero(first)[0]
    vals = v[starts].copy()
    # sequential duplicate sums, in edge order (Synthetic.cpp: vals.back() += v)
    dup = np.nonzero(~first)[0]
    seg = np.searchsorted(starts, dup, side="right") - 1
    for d, s in zip(dup.tolist(), seg.tolist()):
        vals[s] += v[d]
    ukey = key[starts]
    colind = (ukey & np.uint64(0xFFFFFFFF)).astype(np.uint32)
    rows_of = (ukey >> np.uint64(32)).astype(np.int64)
    rowptr = np.zeros(n + 1, dtype=np.uint32)
    rowptr[1:] = np.cumsum(np.bincount(rows_of, minlength=n)).astype(np.uint32)
    return rowptr, colind, vals
