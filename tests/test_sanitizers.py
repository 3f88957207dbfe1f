"""Race / memory-safety checks of the native host runtime.

GPU-side sanitizers are not available on the MI355X pool, so the C++ runtime
(journal, snapshot store, checkpoint writer, CRC32C) is built standalone with
AddressSanitizer + UBSan and, separately, ThreadSanitizer (concurrent journal
appends from 4 threads), and its self-test must pass cleanly under both.  The
actor runtime's single-threaded-mailbox invariant is checked in debug mode."""
import glob
import os
import shutil
import subprocess
import tempfile

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SRC = sorted(glob.glob(os.path.join(ROOT, "csrc", "runtime", "*.cpp")))


def _build_and_run(flags, tmp):
    exe = os.path.join(tmp, "selftest")
    cmd = ["g++", "-std=c++17", "-O1", "-g", "-fno-omit-frame-pointer", *flags, "-o", exe, *SRC, "-lpthread"]
    r = subprocess.run(cmd, capture_output=True, text=True)
    assert r.returncode == 0, r.stderr
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=1:verify_asan_link_order=0",
               UBSAN_OPTIONS="halt_on_error=1", TSAN_OPTIONS="halt_on_error=1")
    out = subprocess.run([exe, os.path.join(tmp, "data")], capture_output=True, text=True, env=env, timeout=300)
    assert out.returncode == 0, out.stdout + out.stderr
    assert "selftest ok" in out.stdout


@pytest.mark.skipif(shutil.which("g++") is None, reason="no g++")
def test_runtime_under_asan_ubsan():
    with tempfile.TemporaryDirectory() as t:
        _build_and_run(["-fsanitize=address,undefined", "-fno-sanitize-recover=all"], t)


@pytest.mark.skipif(shutil.which("g++") is None, reason="no g++")
def test_runtime_under_tsan():
    with tempfile.TemporaryDirectory() as t:
        _build_and_run(["-fsanitize=thread"], t)


def test_actor_debug_mode_detects_off_thread_state_access():
    from sharetrade.actors.runtime import Actor, ActorSystem, Props

    class A(Actor):
        def receive(self, msg):
            if msg == "ok":
                self.context.assert_on_actor_thread()
                self.sender.tell("fine", self.self_ref)

    s = ActorSystem("dbg", debug=True)
    try:
        a = s.actor_of(Props(A))
        assert a.ask("ok", 2).result(3) == "fine"
        cell = a._cell
        with pytest.raises(AssertionError):
            cell.context.assert_on_actor_thread()     # called from the test thread, not the actor's
    finally:
        s.terminate()
