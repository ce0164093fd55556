"""bench.py's algorithmic-byte accounting: the
per-event figures each kernel's roofline divides by, keyed by the kernel labels the
engine's profiler reports."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import bench  # noqa: E402


def test_runs_kernel_bytes_by_table():
    # LA16 tiles (N > 32): 2N read + 4N written; int32 tiles (N <= 32, wide32): 4N + 4N
    assert bench.algorithmic_bytes("(k_la16_rows_runs<int32_t>)", 256, 1000, 900) == 6 * 256 * 1000
    assert bench.algorithmic_bytes("(k_la16_rows_runs<int32_t, true>)", 16, 1000, 900) == 8 * 16 * 1000
    # uint16 runs (N > 128): 2N read + 2N written
    assert bench.algorithmic_bytes("(k_la16_rows_runs<uint16_t>)", 256, 1000, 900) == 4 * 256 * 1000


def test_transpose_and_order_bytes():
    # N <= 16: k_transpose is the FDT -> FD step only
    assert bench.algorithmic_bytes("k_transpose", 16, 1000, 900) == 8 * 16 * 1000
    assert bench.algorithmic_bytes("(k_fd_transpose_ts<int32_t>)", 64, 1000, 900) == 12 * 64 * 1000
    # uint16 runs and FD rows: 2N + 2N + 4N
    assert bench.algorithmic_bytes("(k_fd_transpose_ts<uint16_t>)", 256, 1000, 900) == 8 * 256 * 1000
    # the median: 4N + 48 per ordered event; the rest of the order the 48-byte key
    assert bench.algorithmic_bytes("k_median_wave<4>", 256, 1000, 900) == (4 * 256 + 48) * 900
    assert bench.algorithmic_bytes("k_bucket_sort_all", 256, 1000, 900) == 48 * 900
    # the frontier rows transposed: 8 N^2 per round
    assert bench.algorithmic_bytes("k_witness_la", 256, 1000, 900, rounds=10) == 8 * 256 * 256 * 10
