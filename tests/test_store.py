"""The standalone Store (include/hge.h, babble_amd/csrc/hge_store.cpp): the
reference's store tests -- TestInmemEvents, TestInmemRounds (inmem_store_test.go),
TestParticipantEventsCache(+Edge) (caches_test.go) and the RollingList / LRU
semantics -- restated in C++ against the C ABI (tests/abi/hge_store_test.cpp).
Host only: no device is needed, so this runs in the CPU suite."""
import os
import subprocess

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_store_abi_restated_reference_tests():
    exe = os.path.join(ROOT, "build", "hge_store_test")
    assert os.path.exists(exe), "built by __graft_entry__.build() (tests/abi/Makefile)"
    out = subprocess.run([exe], capture_output=True, text=True, timeout=60)
    assert out.returncode == 0, out.stderr
    assert out.stdout.startswith("ok "), out.stdout
    assert int(out.stdout.split()[1]) > 100


def test_go_shim_logic_replayed_host_part():
    """tests/abi/shim_replay_test.cpp: the Go shim's InmemStore restated in C++ over
    the same calls (key maps, unregistered participants, TestInmemRounds) on the
    standalone store."""
    exe = os.path.join(ROOT, "build", "shim_replay_test")
    assert os.path.exists(exe), "built by __graft_entry__.build() (tests/abi/Makefile)"
    out = subprocess.run([exe], capture_output=True, text=True, timeout=60)
    assert out.returncode == 0, out.stderr + out.stdout
    assert "0 failures" in out.stdout
