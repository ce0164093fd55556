"""Every committed golden (tests/golden/*.npz, oracle outputs made by
tests/golden/make_golden.py) replayed on the HIP engine, all fields bit-exact:
admission status (forks and fork cascades included), order, per-call batches,
Rounds/LCR/LCRE/transactions, undetermined list, every event's round and
witness flag, every witness's fame, every event's roundReceived and every
ordered event's consensus timestamp.

Covers config 5's graph shape (N = 32, 10 forkers, with and without cascades),
the small-N sequential path and the wide path up to 64/100k and 256/51k."""
import glob
import os

import pytest

from parity import compare_golden, load_golden

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GOLDEN = sorted(p for p in glob.glob(os.path.join(ROOT, "tests", "golden", "*.npz"))
                if not os.path.basename(p).startswith("bench_"))


@pytest.mark.parametrize("path", GOLDEN, ids=lambda p: os.path.basename(p))
def test_golden(path):
    from babble_amd.engine import Engine
    dag, g = load_golden(path)
    eng = Engine(int(g["n"]), len(dag["creator"]) + 64)
    try:
        compare_golden(eng, dag, g)
    finally:
        eng.close()
