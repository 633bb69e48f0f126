"""The library's row partition (hipspmv_partition_rows, the one
hipspmv_multi_create cuts with), on the CPU: it depends
only on the matrix -- entries, wcsr segments at the fixed 2^20-column window
(runs of more than 256 entries cut into pieces) and rows -- not on the bench
or on fitted per-matrix weights."""
import numpy as np
import pytest

import hipspmv as hs

LOG2W, CAP, ALIGN = 20, 256, hs.SHARD_ALIGN


def cost_model(rowptr, colind):
    """Per-row cost, restated in numpy: entries + segments + 1."""
    rows = rowptr.size - 1
    lens = np.diff(rowptr.astype(np.int64))
    row_of = np.repeat(np.arange(rows), lens)
    w = colind.astype(np.int64) >> LOG2W
    # a run: consecutive entries of one row in one window
    start = np.ones(colind.size, dtype=bool)
    if colind.size:
        start[1:] = (row_of[1:] != row_of[:-1]) | (w[1:] != w[:-1])
    run_id = np.cumsum(start) - 1
    run_len = np.bincount(run_id)
    run_row = row_of[start]
    seg = np.bincount(run_row, weights=(run_len + CAP - 1) // CAP, minlength=rows)
    return lens + seg + 1


def reference_partition(rowptr, colind, parts):
    cum = np.concatenate([[0.0], np.cumsum(cost_model(rowptr, colind))])
    rows = rowptr.size - 1
    b = [0]
    for p in range(1, parts):
        r = min(int(np.searchsorted(cum, cum[-1] * p / parts, side="left")), rows)
        lo = r // ALIGN * ALIGN
        snap = min(rows, lo if r - lo <= ALIGN // 2 else lo + ALIGN)
        b.append(max(snap, b[-1]))
    return np.array(b + [rows], dtype=np.uint32)


@pytest.mark.parametrize("scale,parts", [(14, 8), (16, 8), (16, 3), (15, 5)])
def test_partition_matches_the_cost_model_on_rmat(scale, parts):
    rowptr, colind, _ = hs.gen_rmat_csr(scale)
    b = hs.partition_rows_cost(rowptr, colind, 1 << scale, parts)
    assert b.tolist() == reference_partition(rowptr, colind, parts).tolist()
    assert b[0] == 0 and b[-1] == 1 << scale and np.all(np.diff(b.astype(np.int64)) >= 0)
    assert np.all(b[1:-1] % ALIGN == 0)


def test_partition_wide_rows_count_their_windows():
    # 3 rows over 2^22 columns: row 0 in one window, row 1 across four, row 2 has 600 entries in one window
    cols = 1 << 22
    r0 = [5, 9]
    r1 = [1, (1 << 20) + 1, (2 << 20) + 1, (3 << 20) + 1]
    r2 = list(range(100, 700))
    colind = np.array(r0 + r1 + r2, dtype=np.uint32)
    rowptr = np.array([0, 2, 6, 606], dtype=np.uint32)
    assert cost_model(rowptr, colind).tolist() == [2 + 1 + 1, 4 + 4 + 1, 600 + 3 + 1]
    assert hs.partition_rows_cost(rowptr, colind, cols, 1).tolist() == [0, 3]


def test_partition_uniform_rows_is_the_entry_balanced_one():
    # equal rows (the stripe matrices C3/C4): cost is proportional to entries
    n = 1 << 14
    rowptr, colind, _ = hs.gen_stripe_csr(0, n, 1 << 21, 32)
    for parts in (2, 4, 8):
        assert hs.partition_rows_cost(rowptr, colind, 1 << 21, parts).tolist() == \
            hs.partition_rows(rowptr, parts).tolist() == [n * p // parts for p in range(parts + 1)]


def test_partition_rejects_bad_input():
    rowptr = np.array([0, 2, 1], dtype=np.uint32)
    colind = np.array([0, 1], dtype=np.uint32)
    with pytest.raises(hs.HipSpMVError):
        hs.partition_rows_cost(rowptr, colind, 4, 2)
    with pytest.raises(hs.HipSpMVError):
        hs.partition_rows_cost(np.array([0, 2], dtype=np.uint32), np.array([0, 9], dtype=np.uint32), 4, 2)
